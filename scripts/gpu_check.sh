#!/bin/bash
# Full GPU test suite (no -x: every failure listed), the default bench line and the per-kernel
# probe, then the N>1 step in a world-1 RCCL group with the bucket sums through RCCL directly
# and through torch's collective.  usage: scripts/gpu_check.sh TAG
set -o pipefail
T=${1:-r04c}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread || exit $?
grep -E "FAILED|ERROR" gpurun_out/$T/pytest_gpu.log | head -20
tail -2 gpurun_out/$T/pytest_gpu.log | head -1
$S 300 gpurun_out/$T/bench.log python bench.py --no-cpu-baseline --no-overlap || exit $?
grep -h '^{' gpurun_out/$T/bench.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['b32']['ms_per_step'], json.dumps(d['roofline']['frac']), json.dumps(d.get('kernel_ms_per_step')))"
for D in 1 0; do
  BA3C_DIRECT_RCCL=$D $S 300 gpurun_out/$T/sync_d$D.log python bench.py --no-cpu-baseline --no-overlap --no-b32 --sync-path || exit $?
  echo -n "direct=$D "
  grep -h '^{' gpurun_out/$T/sync_d$D.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], json.dumps(d['exchange']['timeline']))"
done
# optional same-box A/B: scripts/gpu_check.sh TAG KERNEL LIB...
if [ -n "$2" ]; then
  k=$2; shift 2
  bash scripts/gpu_abk.sh $T/ab $k default "$@"
fi
