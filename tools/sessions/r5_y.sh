#!/bin/bash
# r5 session Y: no trailing barrier per multi-step step (alternating block-sum slots), A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
B="build/ab_old/bin build/bin"
bash tools/variant_ab.sh $O/y_g1.jsonl "miint bench --iters 400" $B > /dev/null && \
bash tools/variant_ab.sh $O/y_s8.jsonl "miint bench --n 1.25e8 --slots 20 --iters 2000" $B > /dev/null && \
bash tools/variant_ab.sh $O/y_s8_48.jsonl "miint bench --n 1.25e8 --slots 48 --iters 2400" $B > /dev/null && \
bash tools/variant_ab.sh $O/y_t2d.jsonl "miint table2d --grid 4096" $B > /dev/null && \
bash tools/variant_ab.sh $O/y_t2d_s8.jsonl "miint table2d --grid 4096 --slice 0/8" $B > /dev/null && \
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $O/y_tests.txt 2>&1
echo "exit $?"
