#!/bin/bash
# r5 session AT: kernel trace of the settled one-shot (one fused launch per integration)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
REPO=$(pwd)
O=$REPO/gpurun_out/r5/at_oneshot
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o os -- \
  python3 $REPO/tools/one_shot_trace.py > $O/os.json 2> $O/os.err
echo "exit $?"
