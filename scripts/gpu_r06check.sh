#!/bin/bash
# HEAD check: the GPU test suite and smoke().
set -o pipefail
T=${1:-r06check}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread && \
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()"
rc=$?
tail -2 gpurun_out/$T/pytest_gpu.log; tail -1 gpurun_out/$T/smoke.log
exit $rc
