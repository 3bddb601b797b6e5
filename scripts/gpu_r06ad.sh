#!/bin/bash
# conv1's and conv2's forward pooled epilogue on the fp32 bits as integers (BA3C_B6_IMAX):
# bit-identity against the committed build, then the same-box A/B (probe: conv1 forward), and
# conv2's forward.
set -o pipefail
T=${1:-r06ad}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
B=distributed-ba3c_amd/ba3c_amd/libba3c_base.so
$S 300 gpurun_out/$T/dump_base.log env BA3C_LIB=$B python scripts/ab_bitident.py dump gpurun_out/$T/base.npz || exit $?
$S 300 gpurun_out/$T/dump_new.log python scripts/ab_bitident.py dump gpurun_out/$T/new.npz || exit $?
python scripts/ab_bitident.py compare gpurun_out/$T/base.npz gpurun_out/$T/new.npz > gpurun_out/$T/cmp.txt 2>&1; tail -3 gpurun_out/$T/cmp.txt
rm -f gpurun_out/$T/*.npz
bash scripts/gpu_abk.sh $T/ab conv1_fwd $B default && \
bash scripts/gpu_abk.sh $T/ab2 conv2_fwd $B default
