#!/usr/bin/env bash
# A/B of 2-D field kernel builds (tile height, read-ahead, full-tile prefetch: the
# MIINT_T2D_* switches of kernels/table.hip, each its own `make cli BUILD=... ABFLAGS=...`)
# across the whole 4096^2 field and its 1/2, 1/4, 1/8 row slices, at 4 and 8 step phases.
# Alternating builds, 2 rounds; one tagged JSON line per run into OUT.
#   tools/t2d_variant_ab.sh OUT.jsonl build/ab_base/bin build/ab_sh30/bin ...
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; shift
mkdir -p "$(dirname "$out")"
: > "$out"
for rep in 1 2; do
  for slice in "" 0/2 0/4 0/8; do
    for ph in ${PHASES:-4 8}; do
      for dir in "$@"; do
        extra=(); [ -n "$slice" ] && extra=(--slice "$slice")
        line=$(timeout -k 10 60 "$dir/miint" table2d --grid 4096 --iters 640 --phases $ph "${extra[@]}" | grep '^{' | tail -1) || {
          echo "{\"build\": \"$dir\", \"failed\": true}" >> "$out"; exit 1; }
        echo "{\"build\": \"$dir\", \"rep\": $rep, \"slice_arg\": \"$slice\", \"phases_arg\": $ph, ${line#\{}" >> "$out"
      done
    done
  done
done
echo "t2d variant A/B: $(wc -l < "$out") runs"
