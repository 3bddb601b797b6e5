#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r04c2
for k in conv2_dgrad conv2_wgrad conv2_fwd; do
  scripts/gpu_step.sh 300 gpurun_out/r04c2/$k.log env BA3C_MULTI_BIG=1 BA3C_BENCH_PROBE=$k python bench.py --no-cpu-baseline --no-overlap --no-b32 || exit $?
  grep -h '^{' gpurun_out/r04c2/$k.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$k', d['ms_per_step'], d['probe'])"
done
