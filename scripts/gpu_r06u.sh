#!/bin/bash
# Diagnostics of the weight-gradient pair launch (timing-only builds, wrong gradients):
# BA3C_DIAG_PAIR=1 runs only the conv0 job, =2 only the conv1 job, against the full pair.
set -o pipefail
T=${1:-r06u}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T conv0_wgrad default $L/libba3c_pd1.so $L/libba3c_pd2.so
