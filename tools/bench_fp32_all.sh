#!/usr/bin/env bash
# bench.py for every integrand in fp32 and fp64 (1 GPU, steady clocks): JSON lines on stdout.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for f in pi4 sin table train poly; do
  for d in fp32 fp64; do
    timeout -k 10 120 python3 bench.py --integrand $f --dtype $d --steps 200 --warmup 10 --no-extras
  done
done
