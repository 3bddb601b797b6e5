#!/bin/bash
# Iteration run: GPU parity tests, the default bench line (B=2048 + configs[1] B=32), then the
# B=32 line under each A/B env given as args.  usage: scripts/gpu_ab32.sh TAG [ENV=VAL ...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
$S 600 gpurun_out/$tag/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
$S 300 gpurun_out/$tag/bench.log python bench.py --no-cpu-baseline --no-overlap && \
for ab in "$@"; do
  $S 200 gpurun_out/$tag/b32_$ab.log env $ab python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 100 --warmup 10 --no-cpu-baseline --no-b32 --no-overlap || exit $?
done
tail -3 gpurun_out/$tag/pytest_gpu.log
grep -h '^{' gpurun_out/$tag/bench.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['value'], d['ms_per_step'], json.dumps(d.get('b32')), json.dumps(d.get('kernel_ms_one_step')))"
for ab in "$@"; do grep -h '^{' gpurun_out/$tag/b32_$ab.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('B=32 $ab', d['value'], d['ms_per_step'], d['ms_per_step_median'])"; done
