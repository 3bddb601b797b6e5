#!/bin/bash
# (1) ba3c_probe_every test; (2) the line's probe bracketing every timed step (--probe-every 1)
# against one step in 5 (the default), alternating; (3) re-tuning sweep of compile-time knobs on
# the round-6 tree: staging loads in flight 8 (BA3C_STAGE_NPT, default 16), conv1 dgrad's ring
# without the next band's register prefetch (BA3C_RING_PRE=0), band MFMA loops at priority 0
# (BA3C_B6_PRIO=0), conv2 weight gradient without A double-buffering (BA3C_W6_DBUF=0), fc1
# backward 3-deep k-tile rings (BA3C_FCD_DEPTH=3), 8 reduction groups (BA3C_RED_GROUPS=8).
set -o pipefail
T=${1:-r06s}
mkdir -p gpurun_out/$T/pe
S=scripts/gpu_step.sh
L=distributed-ba3c_amd/ba3c_amd
$S 300 gpurun_out/$T/pytest_probe.log python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_bench_path.py -k probe_every || exit $?
grep -E "passed|failed" gpurun_out/$T/pytest_probe.log | tail -1
for rep in 1 2; do
  for pe in 1 5; do
    $S 300 gpurun_out/$T/pe/bench_pe${pe}_$rep.log python bench.py --no-cpu-baseline --no-overlap --no-b32 --probe-every $pe || exit $?
  done
done
for f in gpurun_out/$T/pe/*.log; do grep -h '^{' $f | python -c "
import sys,json; d=json.loads(sys.stdin.readline()); print('$f'.split('/')[-1], d['ms_per_step'], d['probe'], d['roofline']['frac'])"; done
bash scripts/gpu_abk.sh $T conv1_dgrad default $L/libba3c_npt8.so $L/libba3c_pre0.so $L/libba3c_prio0.so \
  $L/libba3c_w6dbuf0.so $L/libba3c_fcd3.so $L/libba3c_red8.so
