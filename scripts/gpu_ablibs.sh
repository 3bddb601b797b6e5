#!/bin/bash
# Bench A/B over alternative library builds: scripts/gpu_ablibs.sh TAG lib1.so lib2.so ...
# (each under its own time limit; the default library first)
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
$S 300 gpurun_out/$tag/bench_default.log python bench.py --no-cpu-baseline --no-overlap --no-b32 || exit $?
for lib in "$@"; do
  n=$(basename $lib .so)
  $S 300 gpurun_out/$tag/bench_$n.log env BA3C_LIB=$lib python bench.py --no-cpu-baseline --no-overlap --no-b32 || exit $?
done
for f in gpurun_out/$tag/bench_*.log; do
  echo "$f"; grep -h '^{' $f | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); k=d['kernel_ms_one_step']; print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], {x: k[x] for x in ('conv0_fwd','conv0_wgrad','conv1_fwd','conv1_dgrad','conv1_wgrad')})"
done
