#!/bin/bash
# conv3's whole-image kernels (forward, input gradient) with one persistent workgroup per CU
# (BA3C_C3_WGPC=1: half the weight-fragment loads, twice the images per workgroup) against two.
set -o pipefail
T=${1:-r06z}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/fwd conv3_fwd default $L/libba3c_c3w1.so && \
bash scripts/gpu_abk.sh $T/dg conv3_dgrad default $L/libba3c_c3w1.so
