#!/bin/bash
# 2:4-sparse conv1 weight gradient: the oracle tests that run it (B = 512 hard inputs, B = 2048
# fp64, launch paths), then a same-box A/B of the pair and of conv1's job alone.
set -o pipefail
T=${1:-r05f}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest.log python -u -m pytest -v -s --timeout 240 --timeout-method thread tests/test_gpu_hard_inputs.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_graph.py tests/test_gpu_bench_path.py || exit $?
grep -E "per-tensor|FAILED|ERROR|passed|failed" gpurun_out/$T/pytest.log | head -20
L=distributed-ba3c_amd/ba3c_amd
bash scripts/gpu_abk.sh $T/pair conv0_wgrad default $L/libba3c_dense.so $L/libba3c_diag2.so $L/libba3c_diag2dense.so
