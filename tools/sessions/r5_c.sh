#!/bin/bash
# r5 session C: fused multi-step close A/B (strong shares, headline), series_exact headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python tools/strong_slices.py --gpus 1,8 --steps 20 --collective on --close fused,kernel --jsonl $O/c_close_ab20.jsonl > $O/c_close_ab20.txt 2>&1 && \
timeout -k 10 300 python tools/strong_slices.py --gpus 1,8 --steps 48 --collective on --close fused,kernel --jsonl $O/c_close_ab48.jsonl > $O/c_close_ab48.txt 2>&1 && \
for c in "" "--close-kernel" "" "--close-kernel"; do
  timeout -k 10 200 python bench.py --no-extras --steps 20 --warmup 5 $c >> $O/c_bench20_ab.jsonl 2>> $O/c_bench_ab.err || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_s8f -o s8 --output-format csv -- python3 tools/strong_slices.py --gpus 8 --steps 20 --collective on > $O/c_prof_s8f.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/c_bench20_full.json 2> $O/c_bench20_full.err
echo "exit $?"
