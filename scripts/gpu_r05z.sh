#!/bin/bash
# the whole GPU suite on the tree with the opt-in sparse conv1 input gradient
set -o pipefail
T=${1:-r05z}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread || exit $?
grep -E "rel err|FAILED|ERROR" gpurun_out/$T/pytest_gpu.log | head -20
tail -2 gpurun_out/$T/pytest_gpu.log | head -1
