#!/usr/bin/env bash
# A/B of 2-D field builds of the miint CLI kept under variants/ (miint_*): whole 4096^2 grid
# and one GPU's 1/8 row slice, alternated over passes.
set -e
for pass in 1 2 3; do
  for b in variants/miint_*; do
    for a in "--grid 4096" "--grid 4096 --slice 3/8" "--grid 8192"; do
      printf '%s pass%s %s: ' "$(basename "$b")" "$pass" "$a"
      timeout -k 10 60 "$b" table2d $a --json | grep '^{'
    done
  done
done
