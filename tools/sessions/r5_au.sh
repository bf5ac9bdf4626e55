#!/bin/bash
# r5 session AU: projected strong efficiency at the final build (per-GPU shares of N = 1e9,
# 1-rank RCCL stage, direct batches; 20- and 48-step batches) and the 2-D shares
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
rm -f $O/au_strong20.jsonl $O/au_strong48.jsonl $O/au_t2d.jsonl
timeout -k 10 300 python tools/strong_slices.py --gpus 1,2,4,8 --steps 20 --collective on --graphs off --jsonl $O/au_strong20.jsonl > $O/au_strong20.txt 2>&1 && \
timeout -k 10 300 python tools/strong_slices.py --gpus 1,2,4,8 --steps 48 --collective on --graphs off --jsonl $O/au_strong48.jsonl > $O/au_strong48.txt 2>&1 && \
timeout -k 10 300 python -u tools/t2d_strong.py --collective on --jsonl $O/au_t2d.jsonl > $O/au_t2d.txt 2>&1
echo "exit $?"
