#!/bin/bash
# k-split conv1 band kernels: parity tests, then same-box A/B of conv1 fwd / dgrad against the
# r03 n-block mapping (libba3c_ks0.so) and the k-split without A double buffering (ksnd)
set -o pipefail
T=${1:-r04ks}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
L=distributed-ba3c_amd/ba3c_amd
$S 600 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hard_inputs.py tests/test_gpu_bench_path.py tests/test_gpu_graph.py -x -v --timeout 240 --timeout-method thread || exit $?
tail -2 gpurun_out/$T/pytest_gpu.log
scripts/gpu_abk.sh $T/fwd conv1_fwd default $L/libba3c_ks0.so $L/libba3c_ksnd.so
scripts/gpu_abk.sh $T/dgrad conv1_dgrad default $L/libba3c_ks0.so $L/libba3c_ksnd.so
