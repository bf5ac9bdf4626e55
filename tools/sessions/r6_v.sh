#!/bin/bash
# Round 6, re-entry: validate the rebuilt tree (smoke, the driver's bench line, the GPU suite).
set -o pipefail
O=gpurun_out/v; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gputests.txt 2>&1
rc=$?; echo "rc=$rc"; tail -2 $O/gputests.txt; cat $O/bench.json; exit $rc
