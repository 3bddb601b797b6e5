#!/bin/bash
# fc1's forward k-chunk 320 (5 partial sums for the heads kernel) against 160 (10), at B=2048
# and at configs[1]'s B=32 (the b32 leg), alternating.
set -o pipefail
T=${1:-r06aa}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
for rep in 1 2; do
  for lib in default kc320; do
    if [ $lib = default ]; then ev=(); else ev=(BA3C_LIB=distributed-ba3c_amd/ba3c_amd/libba3c_kc320.so); fi
    $S 300 gpurun_out/$T/bench_${lib}_$rep.log env "${ev[@]}" BA3C_BENCH_PROBE=heads python bench.py --no-cpu-baseline --no-overlap || exit $?
  done
done
for f in gpurun_out/$T/bench_*.log; do grep -h '^{' $f | python -c "
import sys,json; d=json.loads(sys.stdin.readline()); k=d['kernel_ms_per_step']; print('$f'.split('/')[-1], d['ms_per_step'], 'b32', d['b32']['ms_per_step'], d['b32']['ms_per_step_median'], 'fc1f %.1f heads %.1f' % (k['fc1_fwd']*1e3, k['heads']*1e3))"; done
