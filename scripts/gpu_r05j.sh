#!/bin/bash
# conv1 sparse weight gradient with bank-conflict-free B reads (logical quads permuted):
# the oracle tests that run it, then a same-box A/B of the pair against the previous commit.
set -o pipefail
T=${1:-r05j}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest.log python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hard_inputs.py tests/test_gpu_fullsize_oracle.py || exit $?
grep -E "per-tensor|FAILED|ERROR|passed|failed" gpurun_out/$T/pytest.log | head -20
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/pair conv0_wgrad default $L/libba3c_prev.so
