#!/bin/bash
# sparse conv1 input gradient: is the L2 weight-fragment stream the limit? (timing-only build
# that reuses the first k-steps' fragments)
set -o pipefail
T=${1:-r05y}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/c1d conv1_dgrad default $L/libba3c_d1s3.so $L/libba3c_d1s1.so
