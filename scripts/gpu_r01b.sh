set -o pipefail
mkdir -p gpurun_out/r01b
S=scripts/gpu_step.sh
$S 600 gpurun_out/r01b/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread && \
$S 300 gpurun_out/r01b/smoke.log python -c "import __graft_entry__ as g; g.smoke()" && \
$S 300 gpurun_out/r01b/bench.log python bench.py && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
$S 300 gpurun_out/r01b/rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/r01b/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-b32 --no-overlap
echo done
