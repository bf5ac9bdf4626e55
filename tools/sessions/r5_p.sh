#!/bin/bash
# r5 session P: 2-D strong-share rehearsal with the RCCL stage captured (tools/t2d_strong.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
rm -f $O/p_t2d_strong.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_runtime.py -k "table2d" > $O/p_tests.txt 2>&1 || exit 1
timeout -k 10 300 python -u tools/t2d_strong.py --jsonl $O/p_t2d_strong.jsonl > $O/p_t2d_strong.txt 2>&1 && \
timeout -k 10 300 python -u tools/t2d_strong.py --collective on --jsonl $O/p_t2d_strong.jsonl >> $O/p_t2d_strong.txt 2>&1
echo "exit $?"
