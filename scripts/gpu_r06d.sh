#!/bin/bash
# The restructured N>1 step (held fc1 reduction + clip + sum on the exchange stream after the
# phase-2 event): exchange GPU tests, the N=1 line and the world-1 sync path with the --occupy
# table (same box), and a kernel trace of the sync step.
set -o pipefail
T=${1:-r06d}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
Q="--no-cpu-baseline --no-overlap --no-b32"
$S 600 gpurun_out/$T/pytest_x.log python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_bench_path.py tests/test_gpu_replicas.py tests/test_gpu_graph.py || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_x.log | tail -1
for i in 1 2; do
  $S 300 gpurun_out/$T/n1_$i.log python bench.py --no-cpu-baseline --no-overlap || exit $?
  $S 300 gpurun_out/$T/sync_$i.log python bench.py $Q --sync-path --occupy 8,16,32 || exit $?
  for f in n1 sync; do grep -h '^{' gpurun_out/$T/${f}_$i.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$f', d['ms_per_step'], d['ms_per_step_median'], d["device_errors"], d.get("b32",{}).get("ms_per_step"), json.dumps(d.get('exchange',{}).get('timeline')))"; done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$S 300 gpurun_out/$T/trace_sync.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/trace_sync -o run -- python bench.py $Q --sync-path --steps 10 --warmup 2 --occupy 16 || exit $?
