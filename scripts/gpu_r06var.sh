#!/bin/bash
# Box-to-box variance of the final tree: two default-config bench lines (no CPU baseline, no
# configs[4] leg) on whichever box this call gets.
set -o pipefail
T=${1:-r06var}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
for rep in 1 2; do
  $S 300 gpurun_out/$T/bench_$rep.log python bench.py --no-cpu-baseline --no-overlap || exit $?
done
for f in gpurun_out/$T/bench_*.log; do grep -h '^{' $f | python -c "
import sys,json; d=json.loads(sys.stdin.readline()); print('$f'.split('/')[-1], d['ms_per_step'], d['ceiling']['conv_frac_time_weighted'], d['roofline']['frac'], d['b32']['ms_per_step'])"; done
