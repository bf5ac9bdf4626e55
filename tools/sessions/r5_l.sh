#!/bin/bash
# r5 session L: smoke, full GPU tests (verbose), driver-shape bench at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/l_smoke.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/l_gputests.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/l_bench20.json 2> $O/l_bench20.err
echo "exit $?"
