#!/bin/bash
# r5 session X: projected strong efficiency at HEAD (headline shares and 2-D shares, RCCL stage)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
rm -f $O/x_strong20.jsonl $O/x_strong48.jsonl $O/x_t2d_strong.jsonl
timeout -k 10 300 python tools/strong_slices.py --gpus 1,2,4,8 --steps 20 --collective on --jsonl $O/x_strong20.jsonl > $O/x_strong20.txt 2>&1 && \
timeout -k 10 300 python tools/strong_slices.py --gpus 1,2,4,8 --steps 48 --collective on --jsonl $O/x_strong48.jsonl > $O/x_strong48.txt 2>&1 && \
timeout -k 10 300 python -u tools/t2d_strong.py --collective on --jsonl $O/x_t2d_strong.jsonl > $O/x_t2d_strong.txt 2>&1
echo "exit $?"
