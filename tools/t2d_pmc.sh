#!/usr/bin/env bash
# PMC counter groups for the 2-D field kernel alone (one group per rocprofv3 run).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc_t2d
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
G2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY"
G3="FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
G5="TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
for grid in ${T2D_GRIDS:-4096 8192}; do
  for g in G1 G2 G3 G5; do
    timeout -s KILL 60 rocprofv3 --pmc ${!g} --kernel-trace --output-format csv \
      -d "$OUT/t2d_${grid}_$g" -o run -- "$REPO/build/bin/miint" table2d --grid $grid --iters 20 \
      > "$OUT/t2d_${grid}_$g.log" 2>&1
  done
done
echo "pmc done"
