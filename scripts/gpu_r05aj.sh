#!/bin/bash
# conv0's pair workgroups take conv1's last image(s) per CU: parity tests, then a same-box A/B of
# the pair launch (r = 1 default, r = 0 the even split, r = 2)
set -o pipefail
T=${1:-r05aj}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest.log python -u -m pytest tests/test_gpu_fullsize_oracle.py tests/test_gpu_hard_inputs.py -v -s --timeout 300 --timeout-method thread -k "bench_workload or large_batch or ring_walk" || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -3
grep -q " failed" gpurun_out/$T/pytest.log && exit 1
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T conv0_wgrad default $L/libba3c_r0.so $L/libba3c_r2.so
