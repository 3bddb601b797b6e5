#!/bin/bash
# B=2048 step with the large-batch multi-job launches split (BA3C_MULTI_BIG=0, one stream), so
# kernel_ms_per_step shows each job's own time.  usage: scripts/gpu_split2048.sh TAG
set -o pipefail
T=${1:-r04sp}
mkdir -p gpurun_out/$T
BA3C_MULTI_BIG=0 BA3C_OVERLAP=0 scripts/gpu_step.sh 300 gpurun_out/$T/bench_split.log python bench.py --no-cpu-baseline --no-overlap --no-b32 || exit $?
grep -h '^{' gpurun_out/$T/bench_split.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], json.dumps(d['kernel_ms_per_step']))"
