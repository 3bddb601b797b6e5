#!/bin/bash
# GPU parity tests, then the bench (default tree) and any A/B env settings given as args,
# each without the CPU baseline / overlap legs.  usage: scripts/gpu_ab.sh TAG [ENV=VAL ...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
$S 900 gpurun_out/$tag/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread
tail -1 gpurun_out/$tag/pytest_gpu.log
grep -E "^FAILED|^E  " gpurun_out/$tag/pytest_gpu.log | head -20
$S 300 gpurun_out/$tag/bench.log python bench.py --no-cpu-baseline --no-overlap || exit $?
for ab in "$@"; do
  $S 300 gpurun_out/$tag/bench_$ab.log env $ab python bench.py --no-cpu-baseline --no-overlap || exit $?
done
grep -h '^{' gpurun_out/$tag/bench*.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['value'], d['ms_per_step'], d['b32']['value'] if 'b32' in d else '', json.dumps(d.get('kernel_ms_one_step')))"
