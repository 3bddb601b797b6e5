#!/bin/bash
# B=32 kernel trace with the chained reduce -> update (BA3C_DEFER_REDUCE=1): the 12-launch step
set -o pipefail
T=${1:-r05an}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
S=scripts/gpu_step.sh
export BA3C_DEFER_REDUCE=1
$S 300 gpurun_out/$T/rocprof32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32 -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap || exit $?
python scripts/step_timeline.py gpurun_out/$T/stats32/run_kernel_trace.csv 30 > gpurun_out/$T/b32_timeline_defer.txt
cat gpurun_out/$T/b32_timeline_defer.txt | cut -c1-110
