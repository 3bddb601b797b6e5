#!/bin/bash
# conv0 weight gradient with two bands of loads in flight: parity tests, then a same-box A/B of
# the pair launch and of the B=32 step against one band in flight (BA3C_C0W_PFD=1 build)
set -o pipefail
T=${1:-r05ai}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest.log python -u -m pytest tests/test_gpu_fullsize_oracle.py tests/test_gpu_hard_inputs.py tests/test_gpu_graph.py -v -s --timeout 300 --timeout-method thread -k "bench_workload or large_batch or ring_walk or launch_paths or chained" || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -3
grep -q " failed" gpurun_out/$T/pytest.log && exit 1
bash scripts/gpu_abk.sh $T conv0_wgrad default distributed-ba3c_amd/ba3c_amd/libba3c_pfd1.so || exit $?
bash scripts/gpu_ab32.sh $T default distributed-ba3c_amd/ba3c_amd/libba3c_pfd1.so
