#!/bin/bash
# r5 session BA: smoke, full GPU tests (verbose), driver-shape bench at HEAD. The bench runs
# after plain test failures (pytest exit 1), not after a timeout, abort or fault.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/ba_smoke.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/ba_gputests.txt 2>&1
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/ba_bench20.json 2> $O/ba_bench20.err
echo "exit $? (tests $rc)"
