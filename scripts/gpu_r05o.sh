#!/bin/bash
# B=32 kernel timelines (rocprofv3 kernel trace) of this tree and of the previous commit.
set -o pipefail
T=${1:-r05o}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
S=scripts/gpu_step.sh
L=distributed-ba3c_amd/ba3c_amd
$S 300 gpurun_out/$T/rocprof32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32 -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap || exit $?
BA3C_LIB=$L/libba3c_prev.so $S 300 gpurun_out/$T/rocprof32p.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32p -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap || exit $?
python scripts/step_timeline.py gpurun_out/$T/stats32/run_kernel_trace.csv 30
python scripts/step_timeline.py gpurun_out/$T/stats32p/run_kernel_trace.csv 30
