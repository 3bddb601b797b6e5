#!/bin/bash
# The weight-gradient pair's register spill (44 B/lane at 256 VGPRs, from holding the next
# band's X rows through the k-steps): same-box A/B of BA3C_W6S_XPF=1 (default build) vs 0.
set -o pipefail
T=${1:-r06k}
mkdir -p gpurun_out/$T
bash scripts/gpu_abk.sh $T/ab conv0_wgrad default distributed-ba3c_amd/ba3c_amd/libba3c_x1a0.so distributed-ba3c_amd/ba3c_amd/libba3c_x0a0.so
