#!/bin/bash
# fc1's weight-gradient split-K (fewer slabs for the reduction to re-read): same-box A/B of the
# split target, the fc1 backward launch and the step.
set -o pipefail
T=${1:-r06m}
mkdir -p gpurun_out/$T
bash scripts/gpu_abk.sh $T/ab fc1_dgrad default distributed-ba3c_amd/ba3c_amd/libba3c_wt512.so distributed-ba3c_amd/ba3c_amd/libba3c_wt256.so && \
bash scripts/gpu_abk.sh $T/red wgrad_reduce default distributed-ba3c_amd/ba3c_amd/libba3c_wt512.so distributed-ba3c_amd/ba3c_amd/libba3c_wt256.so
