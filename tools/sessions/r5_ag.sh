#!/bin/bash
# r5 session AG: bench with multi-step batches launched directly (default) vs as graph
# replays (--graph-batches), alternating, the driver's exact command (extras on)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
: > $O/ag_bench_ab.jsonl
for rep in 1 2 3 4; do
  for mode in "" "--graph-batches"; do
    timeout -k 10 400 python bench.py --steps 20 --warmup 5 $mode > $O/ag_b.json 2>> $O/ag_bench_ab.err || exit 1
    python3 -c "import json,sys; r=json.loads(open('$O/ag_b.json').read().strip().splitlines()[-1]); print(json.dumps({'mode': '$mode' or 'direct', 'value': r['value'], 'ms_per_step': r['ms_per_step'], 'result': r['result'], 'verified': r['verified'], 'batch_launch': r['config']['batch_launch']}))" >> $O/ag_bench_ab.jsonl
  done
done
echo "exit $?"
