#!/bin/bash
# GPU parity tests only.  usage: scripts/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
T=${1:-r02t}
mkdir -p gpurun_out/$T
if [ -n "$2" ]; then KA=(-k "$2"); else KA=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread "${KA[@]}" > gpurun_out/$T/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/$T/pytest_gpu.log | grep -v "^FAILED\|^ERROR" | sed 's/.*:://' | tr '\n' ' ' | cut -c1-3000
echo; tail -2 gpurun_out/$T/pytest_gpu.log
exit $rc
