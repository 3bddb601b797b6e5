#!/bin/bash
# A/Bs with the registers the round freed: conv2's weight gradient with two k-steps per loop
# iteration (BA3C_W6_UNROLL=2), and the pair's conv1 k-steps at wave priority 1 (BA3C_W6W_PRIO=1).
set -o pipefail
T=${1:-r06l}
mkdir -p gpurun_out/$T
bash scripts/gpu_abk.sh $T/unroll conv2_dgrad default distributed-ba3c_amd/ba3c_amd/libba3c_w6u2.so && \
bash scripts/gpu_abk.sh $T/prio conv0_wgrad default distributed-ba3c_amd/ba3c_amd/libba3c_wprio.so
