#!/bin/bash
# configs[1] (B=32, F=128, S=4) kernel stats: rocprofv3 --kernel-trace --stats of a bench run.
# usage: scripts/gpu_b32prof.sh TAG
set -o pipefail
T=$1
mkdir -p gpurun_out/$T
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32 -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap > gpurun_out/$T/b32.log 2>&1 || exit $?
python scripts/prof_summary.py gpurun_out/$T/stats32/run_kernel_stats.csv | head -40
grep '^{' gpurun_out/$T/b32.log | cut -c1-400
