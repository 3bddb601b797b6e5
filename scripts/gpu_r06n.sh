#!/bin/bash
# conv3's weight gradient riding on conv2's large-batch launch (BA3C_C3W_RIDE 1 / 2) against
# its own launch (0): bit-identity of every output, then the same-box A/B.
set -o pipefail
T=${1:-r06n}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
for r in 0 1 2; do
  $S 300 gpurun_out/$T/dump$r.log env BA3C_C3W_RIDE=$r python scripts/ab_bitident.py dump gpurun_out/$T/ride$r.npz || exit $?
done
python scripts/ab_bitident.py compare gpurun_out/$T/ride0.npz gpurun_out/$T/ride1.npz > gpurun_out/$T/cmp1.txt 2>&1; tail -2 gpurun_out/$T/cmp1.txt
python scripts/ab_bitident.py compare gpurun_out/$T/ride0.npz gpurun_out/$T/ride2.npz > gpurun_out/$T/cmp2.txt 2>&1; tail -2 gpurun_out/$T/cmp2.txt
rm -f gpurun_out/$T/*.npz
bash scripts/gpu_abk.sh $T/ab conv2_dgrad BA3C_C3W_RIDE=0 BA3C_C3W_RIDE=1 BA3C_C3W_RIDE=2
