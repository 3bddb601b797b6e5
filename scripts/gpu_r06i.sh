#!/bin/bash
# Pooled dY staging in wgrad6_body (BA3C_W6_UNPOOL): bit-identity against the per-pixel build,
# the GPU tests of the conv2 / small-batch conv1 weight gradients, and a same-box A/B.
set -o pipefail
T=${1:-r06i}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
$S 300 gpurun_out/$T/dump_a.log python scripts/ab_bitident.py dump gpurun_out/$T/a.npz || exit $?
BA3C_LIB=distributed-ba3c_amd/ba3c_amd/libba3c_w6u0.so $S 300 gpurun_out/$T/dump_b.log python scripts/ab_bitident.py dump gpurun_out/$T/b.npz || exit $?
python scripts/ab_bitident.py compare gpurun_out/$T/a.npz gpurun_out/$T/b.npz | tee gpurun_out/$T/bitident.txt
rm -f gpurun_out/$T/a.npz gpurun_out/$T/b.npz
$S 600 gpurun_out/$T/pytest_x.log python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_path.py tests/test_gpu_graph.py tests/test_gpu_parity.py || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_x.log | tail -1
bash scripts/gpu_abk.sh $T/ab conv2_dgrad default distributed-ba3c_amd/ba3c_amd/libba3c_w6u0.so
