#!/bin/bash
# r5 session AS: per-point accuracy vs speed of the pi4 divisions at the final build
# (384-sample series tiles)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 400 python tools/accuracy_ab.py > $O/as_accuracy_ab.jsonl 2> $O/as_accuracy_ab.err
echo "exit $?"
