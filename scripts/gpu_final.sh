#!/bin/bash
# Round-end check: GPU parity tests, smoke(), full bench line.  usage: scripts/gpu_final.sh TAG
set -o pipefail
T=${1:-r01final}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && \
$S 400 gpurun_out/$T/bench.log python bench.py
tail -2 gpurun_out/$T/pytest_gpu.log; tail -1 gpurun_out/$T/smoke.log; grep '^{' gpurun_out/$T/bench.log
