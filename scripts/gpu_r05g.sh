#!/bin/bash
# Where the sparse conv1 weight gradient's time goes (conv1's job alone in the pair launch):
# full, without the band staging, without the MFMA loop.
set -o pipefail
T=${1:-r05g}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/diag conv0_wgrad $L/libba3c_diag2.so $L/libba3c_d2nostage.so $L/libba3c_d2nomfma.so
