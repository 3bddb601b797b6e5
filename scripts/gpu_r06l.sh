#!/bin/bash
# A/Bs with the registers the round freed: conv2's weight gradient with two k-steps per loop
# iteration (BA3C_W6_UNROLL=2), and the pair's conv1 k-steps at wave priority 1 (BA3C_W6W_PRIO=1).
set -o pipefail
T=${1:-r06l}
mkdir -p gpurun_out/$T
# scripts/gpu_step.sh 300 gpurun_out/$T/pytest_cabi.log python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_bench_path.py -k "cabi or rccl or sync" || exit $?
# grep -E "passed|failed" gpurun_out/$T/pytest_cabi.log | tail -1
bash scripts/gpu_abk.sh $T/unroll conv2_dgrad default distributed-ba3c_amd/ba3c_amd/libba3c_w6u2.so && \
bash scripts/gpu_abk.sh $T/prio conv0_wgrad default distributed-ba3c_amd/ba3c_amd/libba3c_wprio.so
