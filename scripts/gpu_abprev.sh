#!/bin/bash
# Parity tests of the working tree, then same-box A/B of named kernels against libba3c_prev.so
# (scripts/build_prev.sh).  usage: scripts/gpu_abprev.sh TAG "pytest files" KERNEL...
set -o pipefail
T=$1; TESTS=$2; shift 2
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
L=distributed-ba3c_amd/ba3c_amd
if [ -n "$TESTS" ]; then
  $S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest $TESTS -x -v --timeout 240 --timeout-method thread || exit $?
  tail -2 gpurun_out/$T/pytest_gpu.log | head -1
  grep -q " passed" gpurun_out/$T/pytest_gpu.log && ! grep -q "FAILED\|ERROR" gpurun_out/$T/pytest_gpu.log || { grep -E "FAILED|Error" gpurun_out/$T/pytest_gpu.log | head; exit 1; }
fi
for k in "$@"; do
  scripts/gpu_abk.sh $T/$k $k default $L/libba3c_prev.so || exit $?
done
