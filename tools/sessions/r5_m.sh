#!/bin/bash
# r5 session M: 2-D row loop with untied v_fma_f64 line updates (A/B), and the adaptive
# multi-step replay size (build/bin: every switch on + auto replay steps; ab_uo: every
# switch on, 32 integrations per replay)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
B="build/ab_u0/bin build/ab_ub/bin build/ab_uo/bin build/bin"
bash tools/variant_ab.sh $O/m_t2d_full.jsonl "miint table2d --grid 4096" $B > /dev/null && \
bash tools/variant_ab.sh $O/m_t2d_s8.jsonl "miint table2d --grid 4096 --slice 0/8" $B > /dev/null && \
bash tools/variant_ab.sh $O/m_t2d_s4.jsonl "miint table2d --grid 4096 --slice 0/4" $B > /dev/null && \
bash tools/variant_ab.sh $O/m_t2d_s2.jsonl "miint table2d --grid 4096 --slice 0/2" $B > /dev/null && \
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_runtime.py -k "table2d" > $O/m_tests.txt 2>&1
echo "exit $?"
