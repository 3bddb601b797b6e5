#!/bin/bash
# gpu_iter.sh plus the B=32 (configs[1]) bench line.  usage: scripts/gpu_iter_b32.sh TAG
set -o pipefail
tag=$1
bash scripts/gpu_iter.sh $tag || exit $?
timeout -k 10 120 python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap > gpurun_out/$tag/bench_b32.log 2>&1 || exit $?
grep -h '^{' gpurun_out/$tag/bench_b32.log | python -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print('B=32', d['value'], d['ms_per_step'], d['kernel_ms_one_step'].get('fc1_fwd'))"
