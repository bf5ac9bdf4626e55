#!/usr/bin/env bash
# Grid sweep of the multi-step graph batches at the per-GPU shares of the fixed-N headline
# (N = 1e9 over G = 1, 2, 4, 8 GPUs) and of the fp32 path. The auto grid comes from the
# chained policy (~4 tiles per lane below 2.7e8 samples, capped at the multi-step kernel's
# residency); a multi-step batch pays no per-step launch or final reduction, so a larger grid
# may win there. One JSON line per run, tagged {"case": ..., "grid_req": G}.
# Output: gpurun_out/multistep_grid.jsonl. Each run under its own limit; stops at a failure.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/multistep_grid.jsonl
mkdir -p gpurun_out
: > "$out"
run() {  # run CASE GRID ARGS...
  local case=$1 grid=$2; shift 2
  local line
  line=$(timeout -k 10 90 build/bin/miint bench --grid "$grid" "$@" | grep '^{' | tail -1) || {
    echo "{\"case\": \"$case\", \"grid_req\": $grid, \"failed\": true}" >> "$out"; exit 1; }
  echo "{\"case\": \"$case\", \"grid_req\": $grid, ${line#\{}" >> "$out"
}
for rep in 1 2; do
  for g in 0 256 512 768 1024 1280 1536 1792; do
    run share_1_8 $g --integrand pi4 --n 1.25e8 --iters 240 --slots 48
    run share_1_4 $g --integrand pi4 --n 2.5e8 --iters 240 --slots 48
  done
  for g in 0 1024 1536 1792; do
    run share_1_2 $g --integrand pi4 --n 5e8 --iters 192 --slots 48
  done
  for g in 0 1024 1536 1792 2048; do
    run fp32_1e9 $g --integrand pi4 --dtype fp32 --iters 192 --slots 48
  done
done
echo done
