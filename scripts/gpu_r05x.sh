#!/bin/bash
# sparse conv1 input gradient with the single taps in their own LDS array (one read per plane)
set -o pipefail
T=${1:-r05x}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest.log python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_graph.py -k "sparse" || exit $?
grep -E "rel err|FAILED|ERROR|passed|failed" gpurun_out/$T/pytest.log | head
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/c1d conv1_dgrad default $L/libba3c_d1s1.so BA3C_C1D_SPARSE=0
