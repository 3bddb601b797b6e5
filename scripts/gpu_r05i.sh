#!/bin/bash
# Checkpoint of the current tree: the whole GPU suite, smoke, the default bench line, rocprofv3
# stats and the PMC passes.
set -o pipefail
T=${1:-r05i}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread || exit $?
tail -2 gpurun_out/$T/pytest_gpu.log | head -1
grep -E "FAILED|ERROR" gpurun_out/$T/pytest_gpu.log | head
$S 300 gpurun_out/$T/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit $?
tail -1 gpurun_out/$T/smoke.log
$S 300 gpurun_out/$T/bench.log python bench.py --no-cpu-baseline --no-overlap || exit $?
grep -h '^{' gpurun_out/$T/bench.log | python -c "
import sys,json
d=json.loads(sys.stdin.readline()); print(d['value'], d['ms_per_step'], d['b32']['ms_per_step'], d['roofline']['frac'], d['ceiling']); print(json.dumps(d['kernel_ms_per_step']))"
bash scripts/gpu_pmc.sh $T/pmc
