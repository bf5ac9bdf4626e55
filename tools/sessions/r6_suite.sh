#!/bin/bash
# Round 6, re-entry: smoke and the whole GPU suite at the final build.
set -o pipefail
O=gpurun_out/suite; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gputests.txt 2>&1
rc=$?; echo "rc=$rc"; cat $O/smoke.log; tail -2 $O/gputests.txt; exit $rc
