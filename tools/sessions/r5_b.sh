#!/bin/bash
# r5 session B: series_exact (2.5 VALU) accuracy + speed A/B, strong-share fixed costs, tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python tools/accuracy_ab.py > $O/b_accuracy_ab.jsonl 2> $O/b_accuracy_ab.err && \
for d in series series_exact series series_exact; do
  timeout -k 10 200 python bench.py --no-extras --steps 400 --warmup 20 --div $d >> $O/b_div_ab_400.jsonl 2>> $O/b_div_ab.err || exit 1
  timeout -k 10 200 python bench.py --no-extras --steps 20 --warmup 5 --div $d >> $O/b_div_ab_20.jsonl 2>> $O/b_div_ab.err || exit 1
done && \
timeout -k 10 300 python tools/strong_slices.py --gpus 1,2,4,8 --steps 20 --collective on --jsonl $O/b_strong20.jsonl > $O/b_strong20.txt 2>&1 && \
timeout -k 10 300 python tools/strong_slices.py --gpus 1,8 --steps 48 --collective on --jsonl $O/b_strong48.jsonl > $O/b_strong48.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_s8 -o s8 --output-format csv -- python3 tools/strong_slices.py --gpus 8 --steps 20 --collective on > $O/b_prof_s8.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_shared_rccl.py "tests/test_gpu_kernels.py::test_pi4_series_exact_per_point_accuracy" \
  "tests/test_gpu_runtime.py::test_bench_two_ranks_share_one_gpu_over_gloo" \
  "tests/test_gpu_runtime.py::test_bench_two_ranks_shared_gpu_torch_comm" > $O/b_tests.txt 2>&1
echo "exit $?"
