#!/bin/bash
# fc1 forward split-K chunk: 160 (10 chunks, default) against 320 (5) and 800 (2): fewer partial
# sums for the heads kernel to read, fewer and longer workgroups.
set -o pipefail
T=${1:-r06p}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/fc1 fc1_fwd default $L/libba3c_kc320.so $L/libba3c_kc800.so && \
bash scripts/gpu_abk.sh $T/heads heads default $L/libba3c_kc320.so $L/libba3c_kc800.so
