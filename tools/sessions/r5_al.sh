#!/bin/bash
# r5 session AL: final headline records at HEAD (400 steps and the driver's 20), fresh box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/al_bench20.json 2> $O/al_bench20.err && \
timeout -k 10 400 python bench.py > $O/al_bench400.json 2> $O/al_bench400.err
echo "exit $?"
