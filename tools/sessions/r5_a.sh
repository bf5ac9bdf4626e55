#!/bin/bash
# r5 session A: strong-scaling headline at G=1, shared-GPU multi-rank rehearsal, new tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/a_bench20.json 2> $O/a_bench20.err && \
MIINT_OVERSUBSCRIBE=1 timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/a_bench_np2.json 2> $O/a_bench_np2.err && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_shared_rccl.py tests/test_multi_gpu.py \
  "tests/test_gpu_runtime.py::test_cli_riemann_default_is_one_run" \
  "tests/test_gpu_runtime.py::test_cli_riemann_reports_one_shot" \
  "tests/test_gpu_runtime.py::test_cli_riemann_format" \
  tests/test_gpu_runtime.py -k "bench or riemann or one_shot" > $O/a_tests.txt 2>&1
echo "exit $?"
