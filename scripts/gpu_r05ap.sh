#!/bin/bash
# conv1 sparse weight gradient: the half k-step's operands read during the last full step —
# parity tests, then a same-box A/B of the pair against the previous build
set -o pipefail
T=${1:-r05ap}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest.log python -u -m pytest tests/test_gpu_fullsize_oracle.py tests/test_gpu_hard_inputs.py -v -s --timeout 300 --timeout-method thread -k "bench_workload or large_batch or ring_walk" || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -3
grep -q " failed" gpurun_out/$T/pytest.log && exit 1
bash scripts/gpu_abk.sh $T conv0_wgrad default distributed-ba3c_amd/ba3c_amd/libba3c_prevh.so
