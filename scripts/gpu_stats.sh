#!/bin/bash
# rocprofv3 kernel stats only (no counters) of the default bench workload.  usage: scripts/gpu_stats.sh TAG
set -o pipefail
tag=$1
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$tag/stats -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-b32 --no-overlap > gpurun_out/$tag/stats.log 2>&1
echo "stats rc=$?"
grep '^{' gpurun_out/$tag/stats.log | cut -c1-200
