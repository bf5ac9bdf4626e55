#!/usr/bin/env bash
# Fixed per-integration cost: time vs N and launch variants (1 GPU). Output: JSON lines.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { timeout -k 10 120 python bench.py "$@" 2>/dev/null | grep '^{"metric"' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print(json.dumps({'args': '$*', 'N': c['N'], 'ms': d['ms_per_step'], 'value': d['value'], 'grid': c['grid']}))"; }
for n in 1e6 1e7 1e8 3e8 1e9 3e9; do run --samples $n --steps 200; done
run --unfused --steps 200
run --no-graph --steps 200
run --force-collective --steps 200
