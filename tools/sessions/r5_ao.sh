#!/bin/bash
# r5 session AO: auto grid capped at the single-launch kernels' residency — one-shot and
# plan tests, then the driver-shape bench (one integration per call extra)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py -k "grid or one_shot or chained or multistep or riemann or plan" > $O/ao_tests.txt 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/ao_bench20.json 2> $O/ao_bench20.err
echo "exit $?"
