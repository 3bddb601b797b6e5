#!/bin/bash
# B=32 kernel traces of the default build and the small-batch sparse conv1 weight gradient
set -o pipefail
T=${1:-r05ae}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
S=scripts/gpu_step.sh
L=distributed-ba3c_amd/ba3c_amd
for lib in default $L/libba3c_c1ws2.so; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then ev=(); else ev=(BA3C_LIB=$lib); fi
  $S 300 gpurun_out/$T/rocprof32_$n.log env "${ev[@]}" rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/stats32_$n -o run -- python bench.py --batch 32 --fc_neurons 128 --fc_splits 4 --steps 50 --warmup 5 --no-cpu-baseline --no-b32 --no-overlap || exit $?
  python scripts/step_timeline.py gpurun_out/$T/stats32_$n/run_kernel_trace.csv 30 > gpurun_out/$T/timeline_$n.txt
  cat gpurun_out/$T/timeline_$n.txt | cut -c1-120
done
