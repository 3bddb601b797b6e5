#!/bin/bash
# conv0 forward with its chunks software-pipelined: the whole GPU suite, then same-box A/Bs of
# the conv0 forward launch (B=2048) and of the B=32 step against the unpipelined build
set -o pipefail
T=${1:-r05al}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_gpu.log | tail -2
grep -q " failed" gpurun_out/$T/pytest_gpu.log && exit 1
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T conv0_fwd default $L/libba3c_nopipe.so || exit $?
bash scripts/gpu_ab32.sh $T default $L/libba3c_nopipe.so
