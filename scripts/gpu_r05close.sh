#!/bin/bash
# the round's closing tree: the whole GPU suite, smoke and the default bench line
set -o pipefail
T=${1:-r05close}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_gpu.log | tail -1
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -2 gpurun_out/$T/smoke.log | head -1
$S 600 gpurun_out/$T/bench.log python bench.py || exit $?
grep '^{' gpurun_out/$T/bench.log | cut -c1-300
