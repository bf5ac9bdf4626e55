#!/bin/bash
# r5 session AQ: series_exact seed software-pipelined (next tile's seed under this tile's
# pairs) vs not (A/B)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
B="build/bin build/ab_sp/bin"
bash tools/variant_ab.sh $O/aq_g1.jsonl "miint bench --iters 480" $B > /dev/null && \
bash tools/variant_ab.sh $O/aq_s8.jsonl "miint bench --n 1.25e8 --slots 48 --iters 2400" $B > /dev/null && \
bash tools/variant_ab.sh $O/aq_s8_20.jsonl "miint bench --n 1.25e8 --slots 20 --iters 2000" $B > /dev/null && \
bash tools/variant_ab.sh $O/aq_s4.jsonl "miint bench --n 2.5e8 --slots 48 --iters 1200" $B > /dev/null
echo "exit $?"
