set -o pipefail
mkdir -p gpurun_out/r01v6b
S=scripts/gpu_step.sh
$S 600 gpurun_out/r01v6b/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
$S 300 gpurun_out/r01v6b/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && \
$S 400 gpurun_out/r01v6b/bench.log python bench.py
tail -2 gpurun_out/r01v6b/pytest_gpu.log; tail -1 gpurun_out/r01v6b/smoke.log; grep '^{' gpurun_out/r01v6b/bench.log
