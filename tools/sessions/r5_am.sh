#!/bin/bash
# r5 session AM: grid sweep of the 1/8 and 1/4 shares with 384-sample tiles (direct batches)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
rm -f $O/am_grid.jsonl
for rep in 1 2; do
timeout -k 10 300 python tools/strong_slices.py --gpus 4,8 --grids 0,256,512,768,1024,1536,1792 --steps 48 --collective off --graphs off --jsonl $O/am_grid.jsonl > $O/am_grid_$rep.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/strong_slices.py --gpus 1 --grids 0 --steps 48 --collective off --graphs off --jsonl $O/am_grid.jsonl > $O/am_grid_g1.txt 2>&1
echo "exit $?"
