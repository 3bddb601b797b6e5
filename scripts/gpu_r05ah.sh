#!/bin/bash
# conv1 sparse weight gradient with the half k-step: full-size parity tests, then a same-box
# A/B of the pair launch against the padded full k-step (BA3C_W6S_HALF=0 build)
set -o pipefail
T=${1:-r05ah}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest.log python -u -m pytest tests/test_gpu_fullsize_oracle.py tests/test_gpu_hard_inputs.py -v -s --timeout 300 --timeout-method thread -k "fullsize or bench_workload or large_batch or ring_walk" || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -3
grep -q " failed" gpurun_out/$T/pytest.log && exit 1
bash scripts/gpu_abk.sh $T conv0_wgrad default distributed-ba3c_amd/ba3c_amd/libba3c_nohalf.so
