#!/bin/bash
set -o pipefail
T=r04q2
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
BA3C_MULTI=0 scripts/gpu_step.sh 300 gpurun_out/$T/rocprof32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32 -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap
