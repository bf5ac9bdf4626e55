#!/usr/bin/env bash
# bench.py at small N: grid size sweep at 1e6 and 1e8 samples, then the unfused and no-graph
# launch variants. One JSON line per run.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { timeout -k 10 120 python bench.py "$@" 2>/dev/null | grep '^{"metric"' | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['config']
print(json.dumps({'args': '$*', 'N': c['N'], 'us': round(d['ms_per_step']*1e3,2), 'grid': c['grid']}))"; }
for g in 256 512 1024 2048 4096; do run --samples 1e6 --grid $g --steps 200; done
for g in 256 512 1024 2048; do run --samples 1e8 --grid $g --steps 200; done
run --samples 1e8 --unfused --steps 200
run --samples 1e8 --no-graph --steps 200
