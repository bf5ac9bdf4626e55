#!/bin/bash
# Round 6, re-entry: the driver's line (20 steps, 5 warmup) with every extra, and a kernel
# trace of the same line without extras (rocprofv3 --kernel-trace --stats).
set -o pipefail
O=gpurun_out/final; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- \
  python3 bench.py --steps 20 --warmup 5 --no-extras > $O/bench20_trace.json 2> $O/trace.err
rc=$?; echo "rc=$rc"; find $O -name "*stats*"; exit $rc
