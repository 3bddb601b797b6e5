#!/bin/bash
# sparse conv1 input gradient: where the time goes (timing-only builds without staging /
# without the MFMA loop) against the default and the dense ring walk.
set -o pipefail
T=${1:-r05u}
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/c1d conv1_dgrad default $L/libba3c_d1s1.so $L/libba3c_d1s2.so BA3C_C1D_SPARSE=0
