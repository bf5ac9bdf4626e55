#!/usr/bin/env bash
# A/B of multi-step graph batches (one persistent launch per batch; the default) against
# chained batches (one launch per step), for the Riemann kernels and the 2-D field.
# One JSON line per run, tagged {"ab": "multistep"|"chained", "case": ...}.
# Output: gpurun_out/multistep_ab.jsonl. Each run under its own limit; stops at a failure.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/multistep_ab.jsonl
mkdir -p gpurun_out
: > "$out"
run() {  # run CASE TOOL ARGS... : both variants
  local case=$1; shift
  for v in multistep chained; do
    local extra=(); [ $v = chained ] && extra=(--no-multistep)
    local line
    line=$(timeout -k 10 90 build/bin/miint "$@" "${extra[@]}" | grep '^{' | tail -1) || {
      echo "{\"case\": \"$case\", \"ab\": \"$v\", \"failed\": true}" >> "$out"; exit 1; }
    echo "{\"case\": \"$case\", \"ab\": \"$v\", ${line#\{}" >> "$out"
  done
}
for rep in 1 2; do
  run pi4_1e9_k20 bench --integrand pi4 --iters 200 --slots 20
  run pi4_1e9_k48 bench --integrand pi4 --iters 192 --slots 48
  run pi4_1e10_k20 bench --integrand pi4 --n 1e10 --iters 20 --slots 20
  run pi4_share_1_2 bench --integrand pi4 --n 5e8 --iters 200 --slots 20
  run pi4_share_1_4 bench --integrand pi4 --n 2.5e8 --iters 200 --slots 20
  run pi4_share_1_8 bench --integrand pi4 --n 1.25e8 --iters 200 --slots 20
  run pi4_fp32 bench --integrand pi4 --dtype fp32 --iters 200 --slots 20
  run pi4_ieee bench --integrand pi4 --div ieee --iters 40 --slots 20
  run sin bench --integrand sin --iters 200 --slots 20
  run train bench --integrand train --iters 200 --slots 20
  run table bench --integrand table --iters 200 --slots 20  # chained either way (multistep_pays)
  run poly bench --integrand poly --iters 100 --slots 20
  run t2d_4096 table2d --grid 4096
  run t2d_4096_slice_0_8 table2d --grid 4096 --slice 0/8
  run t2d_4096_slice_0_4 table2d --grid 4096 --slice 0/4
  run t2d_4096_slice_0_2 table2d --grid 4096 --slice 0/2
done
echo done
