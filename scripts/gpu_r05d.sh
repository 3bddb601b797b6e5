#!/bin/bash
# fc1 on the gemm6 engine's scaled fp16x3 family: the whole GPU suite, then same-box A/Bs of
# fc1's forward and backward launches and of the step against the previous commit's build.
set -o pipefail
T=${1:-r05d}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread || exit $?
grep -E "per-tensor|FAILED|ERROR" gpurun_out/$T/pytest_gpu.log | head -30
tail -2 gpurun_out/$T/pytest_gpu.log | head -1
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/fwd fc1_fwd default $L/libba3c_prev.so
bash scripts/gpu_abk.sh $T/bwd fc1_dgrad default $L/libba3c_prev.so
bash scripts/gpu_abk.sh $T/heads heads default $L/libba3c_prev.so
