#!/bin/bash
# Same-box A/B of one kernel over library builds, alternating A B .. A B twice:
#   scripts/gpu_abk.sh TAG KERNEL default|lib1.so|ENV=VAL ...
# each run times KERNEL over the 30 timed steps (BA3C_BENCH_PROBE) and prints its average
# launch time and the step throughput.
set -o pipefail
tag=$1; k=$2; shift 2
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    if [ "$lib" = default ]; then ev=();
    elif [[ "$lib" == *=* ]]; then ev=($lib); n=$(echo $lib | tr '=' '_');   # an env setting
    else ev=(BA3C_LIB=$lib); fi
    $S 300 gpurun_out/$tag/bench_${n}_$rep.log env "${ev[@]}" BA3C_BENCH_PROBE=$k python bench.py --no-cpu-baseline --no-overlap --no-b32 || exit $?
  done
done
for f in gpurun_out/$tag/bench_*.log; do
  grep -h '^{' $f | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); r=d['probe']; print('%-40s' % '$f'.split('/')[-1], d['value'], d['ms_per_step'], r['kernel'], r['avg_launch_ms'], (d['roofline'] or {}).get('frac'))"
done
