#!/bin/bash
# conv2 weight gradient alone (large-batch pairs split, one stream) over diagnostic builds.
# usage: scripts/gpu_w6diag.sh TAG LIB...
set -o pipefail
T=$1; shift
mkdir -p gpurun_out/$T
for lib in default "$@"; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then ev=(); else ev=(BA3C_LIB=$lib); fi
  env "${ev[@]}" BA3C_MULTI_BIG=0 BA3C_OVERLAP=0 BA3C_BENCH_PROBE=conv2_wgrad scripts/gpu_step.sh 300 gpurun_out/$T/w6_$n.log python bench.py --no-cpu-baseline --no-overlap --no-b32 || exit $?
  grep -h '^{' gpurun_out/$T/w6_$n.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print('$n', d['ms_per_step'], d['probe'])"
done
