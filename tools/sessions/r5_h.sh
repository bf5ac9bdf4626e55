#!/bin/bash
# r5 session H: batched multi-step block reductions, A/B of the batch size (1 = per step)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
B="build/ab_rb1/bin build/ab_rb2/bin build/ab_rb4/bin"
bash tools/variant_ab.sh $O/h_rb_s8.jsonl "miint bench --integrand pi4 --n 1.25e8 --iters 400 --slots 20" $B > /dev/null && \
bash tools/variant_ab.sh $O/h_rb_s8_k48.jsonl "miint bench --integrand pi4 --n 1.25e8 --iters 480 --slots 48" $B > /dev/null && \
bash tools/variant_ab.sh $O/h_rb_s4.jsonl "miint bench --integrand pi4 --n 2.5e8 --iters 400 --slots 20" $B > /dev/null && \
bash tools/variant_ab.sh $O/h_rb_full.jsonl "miint bench --integrand pi4 --iters 200 --slots 20" $B > /dev/null && \
bash tools/variant_ab.sh $O/h_rb_fp32.jsonl "miint bench --integrand pi4 --dtype fp32 --iters 200 --slots 20" $B > /dev/null && \
bash tools/variant_ab.sh $O/h_rb_sin.jsonl "miint bench --integrand sin --iters 200 --slots 20" $B > /dev/null
echo "exit $?"
