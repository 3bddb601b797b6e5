#!/bin/bash
# Iteration run: GPU parity tests, then the bench (default and any A/B env given as args).
# usage: scripts/gpu_iter.sh TAG [ENV=VAL ...]   (outputs under gpurun_out/TAG/)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
$S 600 gpurun_out/$tag/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
$S 300 gpurun_out/$tag/bench.log python bench.py --no-cpu-baseline --no-overlap && \
for ab in "$@"; do
  $S 300 gpurun_out/$tag/bench_$ab.log env $ab python bench.py --no-cpu-baseline --no-overlap --no-b32 || exit $?
done
tail -3 gpurun_out/$tag/pytest_gpu.log
grep -h '^{' gpurun_out/$tag/bench*.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['value'], d['ms_per_step'], json.dumps(d.get('kernel_ms_one_step')))"
