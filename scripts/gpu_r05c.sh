#!/bin/bash
# conv0 weight gradient's packed-mask un-pooling: the tests that cover it, then a same-box A/B
# of the pair (default vs BA3C_C0W_PKMASK=0) and of conv0's job alone.
set -o pipefail
T=${1:-r05c}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest.log python -u -m pytest -v --timeout 240 --timeout-method thread tests/test_gpu_hard_inputs.py tests/test_gpu_graph.py tests/test_gpu_switches.py tests/test_gpu_parity.py || exit $?
tail -2 gpurun_out/$T/pytest.log | head -1
grep -E "FAILED|ERROR" gpurun_out/$T/pytest.log | head
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/pair conv0_wgrad default $L/libba3c_pk0.so $L/libba3c_diag1.so $L/libba3c_diag1pk0.so
