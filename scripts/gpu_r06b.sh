#!/bin/bash
# Same-box A/B of the event flags (BA3C_EVENTS light vs torch) on the N=1 and the world-1 sync
# step, the --occupy table at high / normal exchange-stream priority, the exchange GPU tests,
# and a kernel trace of the sync step with light events.
set -o pipefail
T=${1:-r06b}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
Q="--no-cpu-baseline --no-overlap --no-b32"
$S 600 gpurun_out/$T/pytest_x.log python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_bench_path.py tests/test_gpu_replicas.py tests/test_gpu_graph.py || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_x.log | tail -1
for E in light torch light torch; do
  BA3C_EVENTS=$E $S 300 gpurun_out/$T/n1_$E.log python bench.py $Q || exit $?
  BA3C_EVENTS=$E $S 300 gpurun_out/$T/sync_$E.log python bench.py $Q --sync-path || exit $?
  for f in n1 sync; do grep -h '^{' gpurun_out/$T/${f}_$E.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$E $f', d['ms_per_step'], d['ms_per_step_median'], json.dumps(d.get('exchange',{}).get('timeline')))"; done
done
$S 300 gpurun_out/$T/occ_hi.log python bench.py $Q --sync-path --occupy 8,16,32 || exit $?
BA3C_XCHG_PRIORITY=0 $S 300 gpurun_out/$T/occ_lo.log python bench.py $Q --sync-path --occupy 16 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$S 300 gpurun_out/$T/trace_sync.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/trace_sync -o run -- python bench.py $Q --sync-path --steps 10 --warmup 2 --occupy 16 || exit $?
$S 300 gpurun_out/$T/trace_n1.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/trace_n1 -o run -- python bench.py $Q --steps 10 --warmup 2 || exit $?
