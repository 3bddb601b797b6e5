#!/bin/bash
# A/B of two builds of libba3c.so in ONE GPU call: the default library vs
# ba3c_amd/libba3c_ab.so (make -C distributed-ba3c_amd ab AB=...), alternated R times
# (bench B=2048 and B=32 each).  usage: scripts/gpu_abl.sh TAG [R]
set -o pipefail
tag=$1; R=${2:-2}
mkdir -p gpurun_out/$tag
S=scripts/gpu_step.sh
AB=$PWD/distributed-ba3c_amd/ba3c_amd/libba3c_ab.so
for r in $(seq 1 $R); do
  for v in A B; do
    if [ $v = B ]; then E="BA3C_LIB=$AB"; else E="BA3C_NOOP=1"; fi
    $S 200 gpurun_out/$tag/big_${v}$r.log env $E python bench.py --steps 30 --no-cpu-baseline --no-b32 --no-overlap || exit $?
    $S 200 gpurun_out/$tag/b32_${v}$r.log env $E python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 200 --warmup 20 --no-cpu-baseline --no-b32 --no-overlap || exit $?
  done
done
for f in gpurun_out/$tag/*.log; do grep -h '^{' $f | python -c "
import sys,json
d=json.loads(sys.stdin.read()); k=d['kernel_ms_one_step']
print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['ms_per_step_median'], json.dumps({x: k[x] for x in ('conv0_fwd','conv1_fwd','conv1_dgrad','conv2_dgrad','conv1_wgrad','heads','fc1_fwd')}))"; done
