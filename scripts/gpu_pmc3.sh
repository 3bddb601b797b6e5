#!/bin/bash
# rocprofv3 kernel stats + PMC passes of the bench workload (one counter group per run, no
# tracing domains mixed with --pmc), each under its own hard time limit.
# usage: scripts/gpu_pmc3.sh TAG [extra env for the bench]
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
CMD="python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-b32 --no-overlap"
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stats -o run -- $CMD > $out/stats.log 2>&1 || { echo "stats rc=$?"; exit 1; }
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 100 rocprofv3 --pmc $ctr --output-format csv -d $out/pmc$i -o run -- $CMD > $out/pmc$i.log 2>&1
  rc=$?
  echo "pmc$i ($ctr) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/pmc$i.log; exit $rc; fi
done
python scripts/pmc_summary.py $out > $out/pmc_summary.txt 2>&1; tail -40 $out/pmc_summary.txt
