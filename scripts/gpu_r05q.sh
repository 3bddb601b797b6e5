#!/bin/bash
# LDS / VALU / MFMA counters of the weight-gradient pair's two halves run alone (timing-only
# builds: BA3C_DIAG_PAIR=1 conv0's job alone, =2 conv1's job alone).
set -o pipefail
T=${1:-r05q}
export TMPDIR=/tmp
L=distributed-ba3c_amd/ba3c_amd
CMD="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-b32 --no-overlap"
for v in pd1 pd2; do
  out=gpurun_out/$T/$v
  mkdir -p $out
  export BA3C_LIB=$L/libba3c_$v.so
  i=2
  for ctr in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
             "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $out/pmc$i -o run -- $CMD > $out/pmc$i.log 2>&1
    rc=$?
    echo "$v pmc$i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $out/pmc$i.log; exit $rc; fi
  done
  python scripts/pmc_summary.py $out | grep -E "kernel|conv0_wgrad"
done
