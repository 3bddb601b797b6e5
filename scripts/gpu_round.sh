#!/bin/bash
# Round check: GPU parity tests, smoke(), the full default bench line, and a rocprofv3 kernel
# stats run of the bench workload.  usage: scripts/gpu_round.sh TAG [pytest -k expr]
set -o pipefail
T=${1:-r02}
K=${2:-}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
if [ -n "$K" ]; then KA=(-k "$K"); else KA=(); fi
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${KA[@]}" && \
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && \
$S 500 gpurun_out/$T/bench.log python bench.py && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
$S 300 gpurun_out/$T/rocprof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-b32 --no-overlap
tail -3 gpurun_out/$T/pytest_gpu.log; tail -1 gpurun_out/$T/smoke.log; grep '^{' gpurun_out/$T/bench.log | cut -c1-1500
cd $GRAFT_REPO_ROOT && $S 300 gpurun_out/$T/rocprof32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32 -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap
