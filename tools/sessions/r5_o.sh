#!/bin/bash
# r5 session O: the adaptive 2-D replay (2^33 samples, auto phases by workgroup count) at
# HEAD: 2-D GPU tests, the whole field and its slices, and the bench record's 2-D extra
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
: > $O/o_t2d.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py -k "table2d" > $O/o_tests.txt 2>&1 || exit 1
for rep in 1 2 3; do
  for sl in "" "--slice 0/2" "--slice 0/4" "--slice 0/8"; do
    timeout -k 10 90 build/bin/miint table2d --grid 4096 $sl | grep '^{' >> $O/o_t2d.jsonl || exit 1
  done
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/o_bench20.json 2> $O/o_bench20.err
echo "exit $?"
