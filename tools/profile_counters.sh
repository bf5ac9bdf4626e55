#!/usr/bin/env bash
# Collect rocprofv3 PMC counters for the hot kernels, one counter group per run
# (--pmc with --kernel-trace only; never combined with sys/runtime traces).
# Output: gpurun_out/pmc/<workload>_<group>/... ; summarise with tools/summarize_counters.py
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp

G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
G2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MUL_F64 SQ_THREAD_CYCLES_VALU"
G3="FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
G4="WRITE_SIZE GRBM_GUI_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_FLAT"
# where a wave's cycles go (waiting on anything / on instruction fetch), for the share vs G = 1
G5="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU GRBM_GUI_ACTIVE"

# ONLY="name1 name2": run just those workloads (default: all)
want() { [ -z "${ONLY:-}" ] || [[ " $ONLY " == *" $1 "* ]]; }
run() {  # name, group-name, counters, command...
  local name=$1 gname=$2 ctrs=$3; shift 3
  want "$name" || return 0
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv \
    -d "$OUT/${name}_${gname}" -o run -- "$@" > "$OUT/${name}_${gname}.log" 2>&1
}

for g in G1 G2; do
  run pi4_series $g "${!g}" "$REPO/build/bin/miint" bench --iters 200 --settle 300
  run pi4_fp32acc $g "${!g}" "$REPO/build/bin/miint" bench --iters 200 --settle 300 --dtype fp32acc
  run sin_fast $g "${!g}" "$REPO/build/bin/miint" bench --iters 40 --settle 40 --integrand sin --div ieee
  run train_fast $g "${!g}" "$REPO/build/bin/miint" bench --iters 40 --settle 40 --integrand train --div ieee
  run table2d_slice8 $g "${!g}" "$REPO/build/bin/miint" table2d --slice 0/8 --iters 2048 --settle-ms 20
  run pi4_ieee $g "${!g}" "$REPO/build/bin/miint" bench --iters 20 --settle 60 --div ieee
  run pi4_fp32 $g "${!g}" "$REPO/build/bin/miint" bench --iters 200 --settle 300 --dtype fp32
  run pi4_series_exact $g "${!g}" "$REPO/build/bin/miint" bench --iters 200 --settle 300 --div series_exact
  # the 1/8 share of the headline (the per-GPU work of an 8-GPU strong step): 20- and 64-step
  # multi-step dispatches (profiles/r6/batch_tail.md)
  run share8_20 $g "${!g}" "$REPO/build/bin/miint" bench --n 1.25e8 --slots 20 --iters 2000 --settle 2000
  run share8_64 $g "${!g}" "$REPO/build/bin/miint" bench --n 1.25e8 --slots 64 --iters 2048 --settle 2048
  run sin $g "${!g}" "$REPO/build/bin/miint" bench --iters 200 --settle 300 --integrand sin
  run sin_ocml $g "${!g}" "$REPO/build/bin/miint" bench --iters 4 --integrand sin --div ieee \
    --trig-library --settle 16
  run train $g "${!g}" "$REPO/build/bin/miint" bench --iters 200 --settle 300 --integrand train
  run poly $g "${!g}" "$REPO/build/bin/miint" bench --iters 100 --settle 200 --integrand poly
  run table $g "${!g}" "$REPO/build/bin/miint" bench --iters 200 --settle 300 --integrand table
  run table2d $g "${!g}" "$REPO/build/bin/miint" table2d --iters 1024 --settle-ms 20
  run dpp_selftest $g "${!g}" python3 "$REPO/tools/dpp_probe.py"
done
# the 2-D field re-stages its table footprint every integration: bytes fetched past L2
for g in G3; do
  run table2d_slice8 $g "${!g}" "$REPO/build/bin/miint" table2d --slice 0/8 --iters 2048 --settle-ms 20
  run table2d $g "${!g}" "$REPO/build/bin/miint" table2d --iters 1024 --settle-ms 20
done
for g in G1 G2 G3 G4; do
  run trainscan $g "${!g}" "$REPO/build/bin/trainscan"
  run materialize $g "${!g}" "$REPO/build/bin/cintegrate" --materialize
done
for g in G5; do
  run g1_w $g "${!g}" "$REPO/build/bin/miint" bench --n 1e9 --slots 20 --iters 400 --settle 400
  run share8_w $g "${!g}" "$REPO/build/bin/miint" bench --n 1.25e8 --slots 20 --iters 2000 --settle 2000
done
echo "pmc done"
