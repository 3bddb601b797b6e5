#!/bin/bash
# GPU parity tests, the default bench line (no CPU baseline) and a B=32 rocprofv3 kernel trace
# (per-step timeline: scripts/step_timeline.py).  usage: scripts/gpu_b32trace.sh TAG [pytest -k expr]
set -o pipefail
T=${1:-r02t}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
if [ -n "$2" ]; then KA=(-k "$2"); else KA=(); fi
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread "${KA[@]}" && \
$S 300 gpurun_out/$T/bench.log python bench.py --no-cpu-baseline --no-overlap && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
$S 300 gpurun_out/$T/rocprof32.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32 -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap
rc=$?
tail -3 gpurun_out/$T/pytest_gpu.log; grep '^{' gpurun_out/$T/bench.log | cut -c1-400; grep -o '"b32".*' gpurun_out/$T/bench.log
exit $rc
