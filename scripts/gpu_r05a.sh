#!/bin/bash
# Round-5 first GPU call: the new B=2048 fp64 test, the per-tensor mean-of-halves, the world-1
# RCCL comm report, the default line, the gloo N=2 rehearsal line, the world-1 sync path and the
# job-alone times of the weight-gradient pair (BA3C_DIAG_PAIR builds).
set -o pipefail
T=${1:-r05a}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 600 gpurun_out/$T/pytest_new.log python -u -m pytest -v -s --timeout 240 --timeout-method thread \
  tests/test_gpu_fullsize_oracle.py tests/test_gpu_predictor.py::test_full_size_gradient_is_batch_mean_of_halves \
  "tests/test_gpu_bench_path.py::test_sync_replicas_rccl_allreduce_world1_equals_single_replica_step" || exit $?
grep -E "per-tensor|passed|failed|FAILED|Error" gpurun_out/$T/pytest_new.log | head -20
$S 300 gpurun_out/$T/bench.log python bench.py --no-cpu-baseline --no-overlap || exit $?
grep -h '^{' gpurun_out/$T/bench.log | cut -c1-400
$S 300 gpurun_out/$T/bench_g2.log python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --no-overlap --no-b32 --steps 10 || exit $?
grep -h '^{' gpurun_out/$T/bench_g2.log | cut -c1-300
$S 300 gpurun_out/$T/sync_d1.log python bench.py --no-cpu-baseline --no-overlap --no-b32 --sync-path || exit $?
bash scripts/gpu_abk.sh $T/pair conv0_wgrad default distributed-ba3c_amd/ba3c_amd/libba3c_diag1.so distributed-ba3c_amd/ba3c_amd/libba3c_diag2.so
