#!/bin/bash
# Round-6 first GPU call: the whole GPU suite (ADVICE r05 fixes), the N=1 line, the world-1
# sync path with the --occupy table, and kernel traces of both steps (same box).
set -o pipefail
T=${1:-r06a}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
Q="--no-cpu-baseline --no-overlap --no-b32"
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_gpu.log | tail -1
$S 300 gpurun_out/$T/bench_n1.log python bench.py $Q || exit $?
grep -h '^{' gpurun_out/$T/bench_n1.log | cut -c1-300
$S 300 gpurun_out/$T/sync_d1.log python bench.py $Q --sync-path --occupy 8,16,32 || exit $?
grep -h '^{' gpurun_out/$T/sync_d1.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$S 300 gpurun_out/$T/trace_sync.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/trace_sync -o run -- python bench.py $Q --sync-path --steps 10 --warmup 2 || exit $?
$S 300 gpurun_out/$T/trace_n1.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/$T/trace_n1 -o run -- python bench.py $Q --steps 10 --warmup 2 || exit $?
find gpurun_out/$T -name "*kernel_trace.csv" | head
