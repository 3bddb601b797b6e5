#!/bin/bash
# same-box A/B of the weight-gradient reduction's slab groups (BA3C_RED_GROUPS 4 / 8 / 16):
# B=2048 and B=32 steps
set -o pipefail
T=${1:-r05ac}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
for rep in 1 2; do
  for lib in default distributed-ba3c_amd/ba3c_amd/libba3c_rg8.so distributed-ba3c_amd/ba3c_amd/libba3c_rg16.so; do
    n=$(basename $lib .so)
    if [ "$lib" = default ]; then ev=(); else ev=(BA3C_LIB=$lib); fi
    $S 300 gpurun_out/$T/bench_${n}_$rep.log env "${ev[@]}" BA3C_BENCH_PROBE=wgrad_reduce python bench.py --steps 30 --no-cpu-baseline --no-overlap || exit $?
  done
done
for f in gpurun_out/$T/bench_*.log; do
  grep -h '^{' $f | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); b=d['b32']; r=d.get('probe') or {}; print('%-26s' % '$f'.split('/')[-1], d['value'], d['ms_per_step'], r.get('avg_launch_ms'), b['ms_per_step'], b.get('ms_per_step_graph'))"
done
