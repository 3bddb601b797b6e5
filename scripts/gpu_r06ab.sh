#!/bin/bash
# Is the kc320 step gain (r06aa) the workspace layout?  fc1's forward partials moved to the end
# of the workspace (BA3C_FCPART_LAST=1: every training buffer 42 MB lower) against the default
# and against the 320 k-chunk build, alternating.
set -o pipefail
T=${1:-r06ab}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T heads default $L/libba3c_fclast.so $L/libba3c_kc320.so
