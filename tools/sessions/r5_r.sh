#!/bin/bash
# r5 session R: 2-D tests after the rank-uniform replay size (incl. the shared-GPU RCCL ranks)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py tests/test_gpu_shared_rccl.py -k "table2d" > $O/r_tests.txt 2>&1
echo "exit $?"
