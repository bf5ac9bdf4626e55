#!/bin/bash
# r5 session E: PMC of the multi-step kernel at the full (1e9) and 1/8-share (1.25e8) sizes,
# and of the in-launch close (fused) against the closing kernel at 1e9
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$PWD
O=$R/gpurun_out/r5/pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
G2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_THREAD_CYCLES_VALU"
run() {  # name group counters args...
  local name=$1 g=$2 c=$3; shift 3
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${name}_$g -o run -- "$R/build/bin/miint" bench "$@" > $O/${name}_$g.log 2>&1
}
for g in G1 G2; do
  run full_kclose $g "${!g}" --iters 96 --settle 300 --close-kernel || exit 1
  run full_fused $g "${!g}" --iters 96 --settle 300 || exit 1
  run s8_kclose $g "${!g}" --n 1.25e8 --iters 400 --settle 1000 --close-kernel || exit 1
  run s8_fused $g "${!g}" --n 1.25e8 --iters 400 --settle 1000 || exit 1
done
echo "pmc done"
