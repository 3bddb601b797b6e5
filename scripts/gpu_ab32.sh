#!/bin/bash
# Same-box A/B of the configs[1] step (B=32, F=128, S=4) over library builds / env settings,
# alternating twice:  scripts/gpu_ab32.sh TAG default|lib.so|ENV=VAL ...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    if [ "$lib" = default ]; then ev=();
    elif [[ "$lib" == *=* ]]; then ev=($lib); n=$(echo $lib | tr '=' '_');
    else ev=(BA3C_LIB=$lib); fi
    $S 300 gpurun_out/$tag/b32_${n}_$rep.log env "${ev[@]}" python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 300 --warmup 30 --no-cpu-baseline --no-overlap --no-b32 || exit $?
  done
done
for f in gpurun_out/$tag/b32_*.log; do
  grep -h '^{' $f | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('%-34s' % '$f'.split('/')[-1], d['value'], d['ms_per_step'], d['ms_per_step_median'])"
done
