#!/bin/bash
# conv1's input gradient on 2:4-sparse MFMA: sparse vs dense, the ring tests, the oracle tests
# that run it (B=512 hard inputs, B=2048 vs float64), then a same-box A/B of the launch.
set -o pipefail
T=${1:-r05t}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 900 gpurun_out/$T/pytest.log python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_hard_inputs.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_parity.py || exit $?
grep -E "rel err|FAILED|ERROR|passed|failed" gpurun_out/$T/pytest.log | head -30
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/c1d conv1_dgrad default $L/libba3c_prev.so
