#!/bin/bash
# r5 session Z: multi-step batches as graph replays vs direct launches (1-rank RCCL stage on/off)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
rm -f $O/z_graphs20.jsonl $O/z_graphs48.jsonl
for rep in 1 2; do
timeout -k 10 300 python tools/strong_slices.py --gpus 1,8 --steps 20 --collective both --graphs both --jsonl $O/z_graphs20.jsonl > $O/z_graphs20_$rep.txt 2>&1 || exit 1
done
timeout -k 10 300 python tools/strong_slices.py --gpus 1,8 --steps 48 --collective both --graphs both --jsonl $O/z_graphs48.jsonl > $O/z_graphs48.txt 2>&1
echo "exit $?"
