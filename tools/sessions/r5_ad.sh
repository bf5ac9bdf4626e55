#!/bin/bash
# r5 session AD: probe — per-wave partials without the per-step barrier (A/B upper bound)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
B="build/bin build/ab_wp/bin"
bash tools/variant_ab.sh $O/ad_s8.jsonl "miint bench --n 1.25e8 --slots 48 --iters 2400" $B > /dev/null && \
bash tools/variant_ab.sh $O/ad_s8_20.jsonl "miint bench --n 1.25e8 --slots 20 --iters 2000" $B > /dev/null && \
bash tools/variant_ab.sh $O/ad_g1.jsonl "miint bench --iters 400" $B > /dev/null
echo "exit $?"
