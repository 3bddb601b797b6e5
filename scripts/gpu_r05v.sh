#!/bin/bash
# sparse conv1 input gradient, whole-image ring walk + A-fragment ring: the tests that run it,
# then A/B against the dense ring walk and a no-staging timing build.
set -o pipefail
T=${1:-r05v}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest.log python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_graph.py -k "sparse or ring" || exit $?
grep -E "rel err|FAILED|ERROR|passed|failed" gpurun_out/$T/pytest.log | head -30
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/c1d conv1_dgrad default BA3C_C1D_SPARSE=0 $L/libba3c_d1s1.so
