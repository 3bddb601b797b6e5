#!/bin/bash
# Round-6 closing measurement of the committed tree: the GPU suite, smoke, the default bench
# line (CPU baseline included), rocprofv3 kernel stats at B=2048 and B=32, the PMC passes.
set -o pipefail
T=${1:-r06final}
bash scripts/gpu_round.sh $T || exit $?
python scripts/step_timeline.py gpurun_out/$T/stats32/run_kernel_trace.csv 30 > gpurun_out/$T/b32_timeline.txt
tail -2 gpurun_out/$T/b32_timeline.txt
bash scripts/gpu_pmc.sh $T/pmc
