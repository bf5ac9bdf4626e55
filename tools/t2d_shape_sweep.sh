#!/usr/bin/env bash
# 2-D field multi-step shape sweep on one build: the whole 4096^2 field and its 1/2, 1/4,
# 1/8 row slices x step phases x rows per wave (forced through --min-wg: 1 = the most rows
# that fit, 16 on 4096^2; one workgroup more than that shape's count = 8 rows; again = 4).
# Alternating, 2 rounds; one tagged JSON line per run into OUT.
#   tools/t2d_shape_sweep.sh OUT.jsonl [build/bin] [phases...]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; bin=${2:-build/bin}; shift 2 || shift $#
phases=("$@"); [ ${#phases[@]} -gt 0 ] || phases=(8 16)
mkdir -p "$(dirname "$out")"
: > "$out"
# workgroups at 16 rows per wave: 1024 / 512 / 256 / 128 for full / 1/2 / 1/4 / 1/8
declare -A nwg=([full]=1024 [0/2]=512 [0/4]=256 [0/8]=128)
for rep in 1 2; do
  for slice in full 0/2 0/4 0/8; do
    n=${nwg[$slice]}
    for mw in 1 $((n + 1)) $((2 * n + 1)); do
      for ph in "${phases[@]}"; do
        extra=(); [ "$slice" != full ] && extra=(--slice "$slice")
        line=$(timeout -k 10 60 "$bin/miint" table2d --grid 4096 --iters 640 --phases "$ph" --min-wg "$mw" "${extra[@]}" | grep '^{' | tail -1) || {
          echo "{\"slice_arg\": \"$slice\", \"failed\": true}" >> "$out"; exit 1; }
        echo "{\"rep\": $rep, \"slice_arg\": \"$slice\", \"phases_arg\": $ph, \"min_wg_arg\": $mw, ${line#\{}" >> "$out"
      done
    done
  done
done
echo "t2d shape sweep: $(wc -l < "$out") runs"
