#!/usr/bin/env bash
# A/B of the 2-D field's multi-step step phases (Table2DConfig::phases, kernels.hpp): one
# workgroup per row-stream block (round 3) against 2 per block (each running every other
# integration of the replay), on the whole 4096^2 field and its 1/2, 1/4, 1/8 row slices
# (the per-GPU share at 2, 4, 8 GPUs). Alternating, 3 rounds. Output:
# gpurun_out/table2d_phases_ab.jsonl (one tagged JSON line per run).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/table2d_phases_ab.jsonl
mkdir -p gpurun_out
: > "$out"
for rep in 1 2 3; do
  for slice in "" 0/2 0/4 0/8; do
    for ph in 1 2; do
      extra=(); [ -n "$slice" ] && extra=(--slice "$slice")
      line=$(timeout -k 10 90 build/bin/miint table2d --grid 4096 --iters 320 --phases $ph "${extra[@]}" | grep '^{' | tail -1) || {
        echo "{\"phases_arg\": $ph, \"slice\": \"$slice\", \"failed\": true}" >> "$out"; exit 1; }
      echo "{\"phases_arg\": $ph, \"rep\": $rep, \"slice_arg\": \"$slice\", ${line#\{}" >> "$out"
    done
  done
done
cat "$out"
