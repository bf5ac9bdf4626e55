#!/bin/bash
# r5 session AI: 384-sample Pi4 series tiles (12 sub-tiles per seed) vs 192 (A/B), then the
# accuracy and bitwise GPU tests of the series paths
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
B="build/ab_t192/bin build/bin"
bash tools/variant_ab.sh $O/ai_g1.jsonl "miint bench --iters 480" $B > /dev/null && \
bash tools/variant_ab.sh $O/ai_g1_series.jsonl "miint bench --iters 480 --div series" $B > /dev/null && \
bash tools/variant_ab.sh $O/ai_s8.jsonl "miint bench --n 1.25e8 --slots 48 --iters 2400" $B > /dev/null && \
bash tools/variant_ab.sh $O/ai_fp32.jsonl "miint bench --iters 480 --dtype fp32" $B > /dev/null && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py tests/test_gpu_runtime.py -k "pi4 or series or multistep or one_shot or bench_contract" > $O/ai_tests.txt 2>&1
echo "exit $?"
