#!/bin/bash
# r5 session AH: kernel trace + stats of the driver-shape bench at HEAD (direct batches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
REPO=$(pwd)
O=$REPO/gpurun_out/r5/ah_prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O -o b20 -- \
  python3 $REPO/bench.py --steps 20 --warmup 5 --no-extras > $O/b20.json 2> $O/b20.err
echo "exit $?"
