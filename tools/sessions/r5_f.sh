#!/bin/bash
# r5 session F: the series_exact headline (closing kernel kept), full GPU tests, bench record
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/f_bench20.json 2> $O/f_bench20.err && \
timeout -k 10 200 python bench.py --no-extras > $O/f_bench400.json 2> $O/f_bench400.err && \
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/f_gputests.txt 2>&1
echo "exit $?"
