#!/usr/bin/env bash
# bench.py for every integrand and path, one JSON line each (profiles/r*/bench_all_integrands.jsonl).
# The first run carries bench.py's extras; the variants skip them (--no-extras).
# Each run under its own time limit; stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { timeout -k 10 120 python bench.py "$@" | grep '^{'; }
run
run() { timeout -k 10 120 python bench.py --no-extras "$@" | grep '^{'; }
run --rule mid
run --div ieee
run --dtype fp32
run --dtype fp32 --rule mid
run --samples 1e10 --steps 100
run --dtype fp32acc
run --integrand sin
run --integrand sin --div ieee
run --integrand train
run --integrand train --div ieee
run --integrand table
run --integrand table --div ieee
run --integrand poly
run --integrand poly --div ieee
