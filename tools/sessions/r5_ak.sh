#!/bin/bash
# r5 session AK: PMC speed of light of the headline kernel (series_exact) at HEAD, its 1/8
# share, the g-fold series, and the driver-shape bench's kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$PWD
O=$R/gpurun_out/r5/pmc_ak
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
G2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU_MUL_F64 SQ_THREAD_CYCLES_VALU GRBM_GUI_ACTIVE"
run() {  # name group counters args...
  local name=$1 g=$2 c=$3; shift 3
  timeout -k 10 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/${name}_$g -o run -- "$R/build/bin/miint" bench "$@" > $O/${name}_$g.log 2>&1
}
for g in G1 G2; do
  run pi4_series_exact $g "${!g}" --iters 192 --settle 300 || exit 1
  run pi4_series_exact_share8 $g "${!g}" --n 1.25e8 --iters 400 --settle 1000 || exit 1
  run pi4_series_g $g "${!g}" --iters 192 --settle 300 --div series || exit 1
done
echo "exit $?"
