#!/bin/bash
# r5 session T: smoke, full GPU tests (verbose), driver-shape bench at HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/t_smoke.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/ > $O/t_gputests.txt 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/t_bench20.json 2> $O/t_bench20.err
echo "exit $?"
