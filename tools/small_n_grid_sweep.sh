#!/usr/bin/env bash
# Grid size vs time per integration at small N (latency-bound regime), 1 GPU.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B=build/bin/miint
for spec in "table 18e6" "table 1e8" "pi4 1e7" "pi4 1e8" "sin 1e7"; do
  set -- $spec
  for g in 128 256 512 1024 2048; do
    echo "{\"integrand\":\"$1\",\"n\":\"$2\",\"grid\":$g,\"row\":$($B bench --integrand $1 --n $2 --grid $g --iters 200 | tail -1)}"
  done
done
