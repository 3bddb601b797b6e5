#!/bin/bash
# Exchange-path GPU tests, then the N>1 step in a world-1 RCCL group (--sync-path) and its
# timeline, with the bucket sums through RCCL directly and through torch's collective.
# usage: scripts/gpu_sync.sh TAG
set -o pipefail
T=${1:-r04s}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest.log python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_replicas.py tests/test_gpu_bench_path.py -x -v --timeout 240 --timeout-method thread || exit $?
tail -2 gpurun_out/$T/pytest.log | head -1
for D in 1 0 1; do
  BA3C_DIRECT_RCCL=$D $S 300 gpurun_out/$T/sync_d$D.log python bench.py --no-cpu-baseline --no-overlap --no-b32 --sync-path || exit $?
  echo -n "direct=$D "
  grep -h '^{' gpurun_out/$T/sync_d$D.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], json.dumps(d['exchange']['timeline']))"
done
