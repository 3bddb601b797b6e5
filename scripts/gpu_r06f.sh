#!/bin/bash
# BA3C_DYNQ A/B after moving the ticket draw off the critical path (atomic inc, drawn after
# the per-image scale): the bit-identity test, then N=1 and world-1 sync lines, DYNQ on / off.
set -o pipefail
T=${1:-r06f}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
Q="--no-cpu-baseline --no-overlap --no-b32"
$S 600 gpurun_out/$T/pytest_x.log python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_graph.py -k "dynamic or ring or two_phase or held" || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_x.log | tail -1
for D in 1 0 1 0; do
  BA3C_DYNQ=$D $S 300 gpurun_out/$T/n1_d$D.log python bench.py $Q || exit $?
  grep -h '^{' gpurun_out/$T/n1_d$D.log | sed "s/^/D$D n1 /" | cut -c1-2000 >> gpurun_out/$T/lines.txt
  BA3C_DYNQ=$D $S 300 gpurun_out/$T/sync_d$D.log python bench.py $Q --sync-path --occupy 16 || exit $?
  grep -h '^{' gpurun_out/$T/sync_d$D.log | sed "s/^/D$D sync /" >> gpurun_out/$T/lines.txt
done
