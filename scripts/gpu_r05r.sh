#!/bin/bash
# conv0 forward epilogue: ReLU count by v_med3_i32 + three-input adds, window max by two
# v_max3_i32 (training block 418 -> 340 VALU per 160 MFMA).  Oracle tests, same-box A/B.
set -o pipefail
T=${1:-r05r}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest.log python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hard_inputs.py tests/test_gpu_graph.py || exit $?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/$T/pytest.log | head -20
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/c0f conv0_fwd default $L/libba3c_prev.so
