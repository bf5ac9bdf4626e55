#!/bin/bash
# r5 session AA: bench with multi-step batches launched directly (default) vs as graph
# replays (--graph-batches), alternating, the driver's shape; then the tests that read the
# record's launch fields
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
: > $O/aa_bench_ab.jsonl
for rep in 1 2 3; do
  for mode in "" "--graph-batches"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras $mode > $O/aa_b.json 2>> $O/aa_bench_ab.err || exit 1
    python3 -c "import json,sys; r=json.loads(open('$O/aa_b.json').read().strip().splitlines()[-1]); print(json.dumps({'mode': '$mode' or 'direct', 'value': r['value'], 'ms_per_step': r['ms_per_step'], 'result': r['result'], 'verified': r['verified'], 'batch_launch': r['config']['batch_launch']}))" >> $O/aa_bench_ab.jsonl
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_runtime.py tests/test_gpu_shared_rccl.py tests/test_scaling_gpu.py -k "bench or scale" > $O/aa_tests.txt 2>&1
echo "exit $?"
