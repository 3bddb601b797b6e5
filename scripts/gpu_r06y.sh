#!/bin/bash
# Diagnostic (timing-only build, wrong outputs): the band kernels' pooled epilogue without its
# global stores (BA3C_DIAG_NOEPI=1) — what the per-lane dword + byte stores of conv1's and
# conv2's forward cost.
set -o pipefail
T=${1:-r06y}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T conv1_fwd default $L/libba3c_noepi.so
