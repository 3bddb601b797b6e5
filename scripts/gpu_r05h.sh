#!/bin/bash
# 2:4-sparse conv0 weight gradient: the 16x16x32 sparse-MFMA probe, the oracle tests that run
# conv0's weight gradient (small and large batch), then a same-box A/B of the pair and of
# conv0's job alone.
set -o pipefail
T=${1:-r05h}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 120 gpurun_out/$T/probe.log scripts/probes/smfmac_probe || exit $?
grep -E "16x16x32|smfmac" gpurun_out/$T/probe.log
$S 600 gpurun_out/$T/pytest.log python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_hard_inputs.py tests/test_gpu_fullsize_oracle.py || exit $?
grep -E "per-tensor|FAILED|ERROR|passed|failed" gpurun_out/$T/pytest.log | head -20
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/pair conv0_wgrad default $L/libba3c_c0dense.so $L/libba3c_diag1.so $L/libba3c_diag1dense.so
