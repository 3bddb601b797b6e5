#!/bin/bash
# Same-box comparison of the closing tree (default) against the round's previous closing tree
# (commit a13f6ef, profiles r06final3: libba3c_prev.so), three alternating pairs.
set -o pipefail
T=${1:-r06x}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
for rep in 1 2 3; do
  for lib in default prev; do
    if [ $lib = default ]; then ev=(); else ev=(BA3C_LIB=distributed-ba3c_amd/ba3c_amd/libba3c_prev.so); fi
    $S 300 gpurun_out/$T/bench_${lib}_$rep.log env "${ev[@]}" python bench.py --no-cpu-baseline --no-overlap --no-b32 || exit $?
  done
done
for f in gpurun_out/$T/bench_*.log; do grep -h '^{' $f | python -c "
import sys,json; d=json.loads(sys.stdin.readline()); print('$f'.split('/')[-1], d['ms_per_step'], d['ceiling']['conv_frac_time_weighted'], d['roofline']['frac'])"; done
