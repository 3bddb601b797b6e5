#!/bin/bash
# Quick iteration: selected GPU tests (pytest -k expression, or all with "all"), then same-box
# A/B probes of kernels over library builds.
# usage: scripts/gpu_quick.sh TAG "KEXPR|all" "KERNEL[,KERNEL...]" LIB...
set -o pipefail
T=$1; K=$2; KS=$3; shift 3
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
if [ "$K" = all ]; then KA=(); else KA=(-k "$K"); fi
$S 600 gpurun_out/$T/pytest_gpu.log python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread "${KA[@]}" || exit $?
grep -E "FAILED|ERROR" gpurun_out/$T/pytest_gpu.log | head -20
tail -2 gpurun_out/$T/pytest_gpu.log | head -1
for k in ${KS//,/ }; do
  bash scripts/gpu_abk.sh $T/ab_$k $k default "$@" || exit $?
done
