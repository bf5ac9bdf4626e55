#!/usr/bin/env bash
# 2-D field (BASELINE #5): whole-grid and per-GPU row-slice times at 4096^2 and 8192^2,
# one JSON line each (profiles/r1/table2d_slices.jsonl).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for g in 4096 8192; do
  timeout -k 10 60 build/bin/miint table2d --grid $g --iters 200
  for w in 2 4 8; do timeout -k 10 60 build/bin/miint table2d --grid $g --slice 1/$w --iters 200; done
done
