#!/bin/bash
# Full GPU suite on the current tree, then a same-box A/B of the weight-gradient pair:
# default (balanced units, lookahead 1), the old tap partition, lookahead 2, and conv1's job
# alone (BA3C_DIAG_PAIR=2) at lookahead 1 / 2.
set -o pipefail
T=${1:-r05b}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread || exit $?
grep -E "per-tensor|FAILED|ERROR" gpurun_out/$T/pytest_gpu.log | head -20
tail -2 gpurun_out/$T/pytest_gpu.log | head -1
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/pair conv0_wgrad default $L/libba3c_bal0.so $L/libba3c_pf2.so $L/libba3c_diag2.so $L/libba3c_diag2pf2.so
