#!/bin/bash
# fc1's large-batch backward on 128 x 128 tiles (BA3C_FC1_BIGTILE, 5 weight-gradient slabs):
# the parity tests that run it (B=160 bench geometry, B=2048 every gradient against float64,
# the switches at B=160), then the same-box A/B against the committed build (probe: the fc1
# backward launch).
set -o pipefail
T=${1:-r06v}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
B=distributed-ba3c_amd/ba3c_amd/libba3c_base.so
$S 600 gpurun_out/$T/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_bench_path.py tests/test_gpu_fullsize_oracle.py tests/test_gpu_switches.py || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -1
bash scripts/gpu_abk.sh $T/ab fc1_dgrad $B default && \
  bash scripts/gpu_abk.sh $T/abf fc1_fwd default distributed-ba3c_amd/ba3c_amd/libba3c_f1f.so
