#!/usr/bin/env bash
# A/B of kernel variants, each its own CLI build (a variant is a temporary -D switch in the
# kernel source, built with `make cli BUILD=build/ab_<name> ABFLAGS=-D<SWITCH>=<v>`):
#
#   tools/variant_ab.sh OUT.jsonl "miint bench --integrand pi4 --dtype fp32 --iters 192" \
#       build/bin build/ab_a/bin build/ab_b/bin
#
# Runs `<dir>/<program> <args>` (the first word names the tool) for every build dir in turn, 3 rounds (alternating, so clock and
# thermal drift hits every variant alike), one tagged JSON line per run into OUT.
# (Round 4's fp32 two-running-sums A/B: profiles/r4/fp32_ab.md.)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1 args=$2; shift 2
mkdir -p "$(dirname "$out")"
: > "$out"
for rep in 1 2 3; do
  for dir in "$@"; do
    # shellcheck disable=SC2086
    line=$(timeout -k 10 90 "$dir/"$args | grep '^{' | tail -1) || {
      echo "{\"build\": \"$dir\", \"failed\": true}" >> "$out"; exit 1; }
    echo "{\"build\": \"$dir\", \"rep\": $rep, ${line#\{}" >> "$out"
  done
done
cat "$out"
