#!/bin/bash
# fc1's large-batch backward on 128 x 128 tiles with 3- and 4-deep k-tile register rings
# (BA3C_FCD_DEPTH) against 2 (the default) and the committed 64 x 64 build (base).
set -o pipefail
T=${1:-r06w}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T fc1_dgrad default $L/libba3c_fd3.so $L/libba3c_fd4.so $L/libba3c_base.so
