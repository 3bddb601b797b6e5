#!/bin/bash
# Chained launches: cost of the per-workgroup release / acquire (timing-only build without
# them) against the unchained previous commit.
set -o pipefail
T=${1:-r05l}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
L=distributed-ba3c_amd/ba3c_amd
for rep in 1 2; do
  for lib in default $L/libba3c_nofence.so $L/libba3c_prev.so; do
    n=$(basename $lib .so)
    if [ "$lib" = default ]; then ev=(); else ev=(BA3C_LIB=$lib); fi
    $S 300 gpurun_out/$T/bench_${n}_$rep.log env "${ev[@]}" python bench.py --no-cpu-baseline --no-overlap --steps 30 || exit $?
  done
done
for f in gpurun_out/$T/bench_*.log; do
  grep -h '^{' $f | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); b=d['b32']; print('%-36s' % '$f'.split('/')[-1], d['value'], d['ms_per_step'], 'b32', b['ms_per_step'], b['ms_per_step_median'], b.get('ms_per_step_graph'), json.dumps({k: d['kernel_ms_per_step'][k] for k in ('conv0_fwd','fc1_fwd','heads')}))"
done
