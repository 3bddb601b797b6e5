#!/bin/bash
# A/B of environment settings: bench line + one LDS/SQ PMC pass per setting.
# usage: scripts/gpu_envpmc.sh TAG ENV=VAL ...   (outputs under gpurun_out/TAG/)
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
CMD="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-b32 --no-overlap"
for ab in "$@"; do
  timeout -k 10 300 env $ab python bench.py --no-cpu-baseline --no-overlap --no-b32 > $out/bench_$ab.log 2>&1 || { echo "bench $ab rc=$?"; exit 1; }
  grep -h '^{' $out/bench_$ab.log | python -c "
import sys,json
d=json.loads(sys.stdin.read()); print('$ab', d['value'], d['ms_per_step'], json.dumps(d.get('kernel_ms_one_step')))"
  export $ab
  timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/pmc_$ab -o run -- $CMD > $out/pmc_$ab.log 2>&1 || { echo "pmc $ab rc=$?"; tail -3 $out/pmc_$ab.log; exit 1; }
  unset ${ab%%=*}
done
