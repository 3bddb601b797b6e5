#!/bin/bash
# B=32 (configs[1]) per-kernel profile: bench at --batch 32 under rocprofv3 --kernel-trace --stats.
set -o pipefail
tag=$1
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 120 python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap > gpurun_out/$tag/bench_b32.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/stats -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 20 --warmup 2 --no-cpu-baseline --no-b32 --no-overlap > gpurun_out/$tag/stats.log 2>&1
echo rc=$?
grep '^{' gpurun_out/$tag/bench_b32.log | cut -c1-400
