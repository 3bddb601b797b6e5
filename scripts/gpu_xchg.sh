#!/bin/bash
# Exchange-path check on one GPU: N=1 bench, the N>1 step in a world-1 RCCL group
# (--sync-path), two ranks started by bench.py itself (no torchrun, gloo rehearsal), the same
# under torchrun, and the replica GPU tests.  usage: scripts/gpu_xchg.sh TAG
set -o pipefail
T=${1:-r04x}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
Q="--no-cpu-baseline --no-overlap"
$S 300 gpurun_out/$T/bench_n1.log python bench.py $Q && \
$S 300 gpurun_out/$T/bench_sync1.log python bench.py $Q --no-b32 --sync-path && \
$S 300 gpurun_out/$T/bench_g2.log python bench.py $Q --no-b32 --gpus 2 --dist-backend gloo --steps 10 --warmup 2 && \
$S 300 gpurun_out/$T/bench_g2_torchrun.log python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py $Q --no-b32 --gpus 2 --dist-backend gloo --steps 10 --warmup 2 && \
$S 600 gpurun_out/$T/pytest_replicas.log python -u -m pytest tests/test_gpu_replicas.py tests/test_gpu_graph.py -x -v --timeout 240 --timeout-method thread
for f in gpurun_out/$T/*.log; do echo "== $f"; grep -h '^{' $f | cut -c1-400; tail -2 $f; done
