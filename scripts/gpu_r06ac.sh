#!/bin/bash
# fc1's forward in 5 k-chunks of two 5-tile halves (BA3C_FC_HALVES): the parity and
# batch-independence tests, then the same-box A/B (B=2048 line and the B=32 leg) against the
# committed 10-chunk build.
set -o pipefail
T=${1:-r06ac}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
B=distributed-ba3c_amd/ba3c_amd/libba3c_base.so
$S 900 gpurun_out/$T/pytest.log python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_gpu_predictor.py tests/test_gpu_parity.py tests/test_gpu_bench_path.py tests/test_gpu_switches.py \
  tests/test_gpu_graph.py || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest.log | tail -1
for rep in 1 2; do
  for lib in default base; do
    if [ $lib = default ]; then ev=(); else ev=(BA3C_LIB=$B); fi
    $S 300 gpurun_out/$T/bench_${lib}_$rep.log env "${ev[@]}" BA3C_BENCH_PROBE=heads python bench.py --no-cpu-baseline --no-overlap || exit $?
  done
done
for f in gpurun_out/$T/bench_*.log; do grep -h '^{' $f | python -c "
import sys,json; d=json.loads(sys.stdin.readline()); k=d['kernel_ms_per_step']; print('$f'.split('/')[-1], d['ms_per_step'], 'b32', d['b32']['ms_per_step'], d['b32']['ms_per_step_median'], 'fc1f %.1f heads %.1f' % (k['fc1_fwd']*1e3, k['heads']*1e3))"; done
