#!/bin/bash
# Same-box A/Bs: conv0 wgrad's frame-first LDS (pair), wave priority 1 around the MFMA loops of
# conv1's weight gradient (pair) and of the band kernels (conv1 forward / input gradient).
set -o pipefail
T=${1:-r05e}
mkdir -p gpurun_out/$T
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/pair conv0_wgrad default $L/libba3c_xf0.so $L/libba3c_w6prio.so || exit $?
bash scripts/gpu_abk.sh $T/c1f conv1_fwd default $L/libba3c_b6prio.so || exit $?
bash scripts/gpu_abk.sh $T/c1d conv1_dgrad default $L/libba3c_b6prio.so
