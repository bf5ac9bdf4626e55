#!/usr/bin/env bash
# Trainscan kernels: LDS counters and kernel-trace stats for each algorithm.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for algo in onepass fused; do
  timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$OUT/ts_$algo" -o run -- "$REPO/build/bin/trainscan" --algo $algo --iters 20 > "$OUT/ts_$algo.log" 2>&1
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ts_stats_$algo" -o run -- "$REPO/build/bin/trainscan" --algo $algo --iters 50 > "$OUT/ts_stats_$algo.log" 2>&1
done
echo ok
