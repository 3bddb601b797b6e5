#!/bin/bash
# Dynamic image queue of the ring walks (BA3C_DYNQ): GPU tests, then same-box N=1 and world-1
# sync lines with the --occupy table, DYNQ on and off.
set -o pipefail
T=${1:-r06e}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
Q="--no-cpu-baseline --no-overlap --no-b32"
$S 900 gpurun_out/$T/pytest_x.log python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_graph.py tests/test_gpu_switches.py tests/test_gpu_hard_inputs.py tests/test_gpu_bench_path.py tests/test_gpu_replicas.py tests/test_gpu_fullsize_oracle.py || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_x.log | tail -1
grep -E "flips vs|model bound|sparse vs dense" gpurun_out/$T/pytest_x.log
for D in 1 0 1 0; do
  BA3C_DYNQ=$D $S 300 gpurun_out/$T/n1_d$D.log python bench.py $Q || exit $?
  BA3C_DYNQ=$D $S 300 gpurun_out/$T/sync_d$D.log python bench.py $Q --sync-path --occupy 16,32 || exit $?
  cat gpurun_out/$T/n1_d$D.log gpurun_out/$T/sync_d$D.log | grep -h '^{' | cut -c1-200 >> gpurun_out/$T/lines.txt
done
