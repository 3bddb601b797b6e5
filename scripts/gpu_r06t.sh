#!/bin/bash
# fc1 and head weight gradients with the XCD-grouped tile order (ba3c_multi.h xcd_group):
# bit-identity against the committed build, then the same-box A/B (probe: fc1 backward launch).
set -o pipefail
T=${1:-r06t}
mkdir -p gpurun_out/$T
S=scripts/gpu_step.sh
B=distributed-ba3c_amd/ba3c_amd/libba3c_base.so
$S 300 gpurun_out/$T/dump_base.log env BA3C_LIB=$B python scripts/ab_bitident.py dump gpurun_out/$T/base.npz || exit $?
$S 300 gpurun_out/$T/dump_new.log python scripts/ab_bitident.py dump gpurun_out/$T/new.npz || exit $?
python scripts/ab_bitident.py compare gpurun_out/$T/base.npz gpurun_out/$T/new.npz > gpurun_out/$T/cmp.txt 2>&1; tail -3 gpurun_out/$T/cmp.txt
rm -f gpurun_out/$T/*.npz
bash scripts/gpu_abk.sh $T/ab fc1_dgrad $B default
