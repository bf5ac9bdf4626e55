#!/bin/bash
# r5 session D: designated-closer multi-step close A/B (strong shares, headline), series_exact headline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python tools/strong_slices.py --gpus 1,8 --steps 20 --collective on --close fused,kernel --jsonl $O/d_close_ab20.jsonl > $O/d_close_ab20.txt 2>&1 && \
timeout -k 10 300 python tools/strong_slices.py --gpus 1,8 --steps 48 --collective on --close fused,kernel --jsonl $O/d_close_ab48.jsonl > $O/d_close_ab48.txt 2>&1 && \
for c in "" "--close-kernel" "" "--close-kernel"; do
  timeout -k 10 200 python bench.py --no-extras --steps 20 --warmup 5 $c >> $O/d_bench20_ab.jsonl 2>> $O/d_bench_ab.err || exit 1
done && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_s8d -o s8 --output-format csv -- python3 tools/strong_slices.py --gpus 8 --steps 20 --collective on > $O/d_prof_s8d.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/d_bench20_full.json 2> $O/d_bench20_full.err
echo "exit $?"
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_gpu_kernels.py tests/test_gpu_runtime.py > $O/d_tests.txt 2>&1
echo "tests exit $?"
