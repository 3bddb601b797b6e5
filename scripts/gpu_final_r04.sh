#!/bin/bash
# Round-4 closing evidence in one call: every GPU test, smoke(), the default bench line (CPU
# baseline included), rocprofv3 kernel stats at B=2048 and B=32, and the PMC passes.
# usage: scripts/gpu_final_r04.sh TAG
set -o pipefail
T=${1:-r04final}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit $?
tail -2 gpurun_out/$T/pytest_gpu.log
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
$S 400 gpurun_out/$T/bench.log python bench.py || exit $?
grep '^{' gpurun_out/$T/bench.log | cut -c1-300
bash scripts/gpu_prof32.sh $T || exit $?
bash scripts/gpu_pmc.sh $T/pmc || exit $?
