#!/bin/bash
# rocprofv3 kernel stats of the configs[1] step (B=32) and of the bench step (B=2048).
# usage: scripts/gpu_prof32.sh TAG
set -o pipefail
T=${1:-r04p}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/$T/rocprof32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32 -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap || exit $?
$S 300 gpurun_out/$T/rocprof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-b32 --no-overlap || exit $?
