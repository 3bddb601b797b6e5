#!/bin/bash
# conv0's chained launch (self-split fragments, late wait for the zeroing): tests, same-box
# A/B of both steps against the previous commit, the B=32 kernel timeline.
set -o pipefail
T=${1:-r05p}
bash scripts/gpu_r05k.sh $T || exit $?
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/$T/rocprof32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32 -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap || exit $?
python scripts/step_timeline.py gpurun_out/$T/stats32/run_kernel_trace.csv 30
