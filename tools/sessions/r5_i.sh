#!/bin/bash
# r5 session I: series_exact tiles with two running e^2 sums (A/B), and the 1/8 share's grid
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
B="build/ab_ts0/bin build/ab_ts1/bin"
bash tools/variant_ab.sh $O/i_ts_s8.jsonl "miint bench --integrand pi4 --n 1.25e8 --iters 400 --slots 20" $B > /dev/null && \
bash tools/variant_ab.sh $O/i_ts_s8_g256.jsonl "miint bench --integrand pi4 --n 1.25e8 --iters 400 --slots 20 --grid 256" $B > /dev/null && \
bash tools/variant_ab.sh $O/i_ts_s4.jsonl "miint bench --integrand pi4 --n 2.5e8 --iters 400 --slots 20" $B > /dev/null && \
bash tools/variant_ab.sh $O/i_ts_full.jsonl "miint bench --integrand pi4 --iters 200 --slots 20" $B > /dev/null && \
bash tools/variant_ab.sh $O/i_ts_full48.jsonl "miint bench --integrand pi4 --iters 192 --slots 48" $B > /dev/null
echo "exit $?"
