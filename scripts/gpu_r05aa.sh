#!/bin/bash
# reduce -> clip + update as one chained launch (phase 3): graph tests, then a same-box A/B of
# the B=32 and B=2048 steps against BA3C_DEFER_REDUCE=0
set -o pipefail
T=${1:-r05aa}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest_graph.log python -u -m pytest tests/test_gpu_graph.py -v -s --timeout 300 --timeout-method thread || exit $?
grep -E "passed|failed|FAILED|ERROR" gpurun_out/$T/pytest_graph.log | tail -5
grep -q " failed" gpurun_out/$T/pytest_graph.log && exit 1
for rep in 1 2; do
  for d in 0 1; do
    $S 300 gpurun_out/$T/bench_d${d}_$rep.log env BA3C_DEFER_REDUCE=$d python bench.py --steps 30 --no-cpu-baseline --no-overlap || exit $?
  done
done
for f in gpurun_out/$T/bench_*.log; do
  grep -h '^{' $f | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); b=d['b32']; print('%-22s' % '$f'.split('/')[-1], d['value'], d['ms_per_step'], b['ms_per_step'], b.get('ms_per_step_graph'), b.get('device_errors', 0))"
done
