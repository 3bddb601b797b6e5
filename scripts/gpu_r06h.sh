#!/bin/bash
# configs[4] partition variants (predictor on a CU-masked stream) and their bit-identity test,
# the DYNQ=1 switch tests, and the default line with overlap and B=32.
set -o pipefail
T=${1:-r06h}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest_x.log python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_path.py tests/test_gpu_switches.py || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_x.log | tail -1
$S 400 gpurun_out/$T/bench.log python bench.py --no-cpu-baseline || exit $?
grep -h '^{' gpurun_out/$T/bench.log | python -c "import sys,json; d=json.loads(sys.stdin.readline()); print(d['ms_per_step'], json.dumps(d['overlap']), json.dumps(d['b32']))"
