#!/bin/bash
# r5 session AW: the driver's bench line three times on one box (box-to-box spread evidence)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras > $O/aw_b.json 2>/dev/null || exit 1
  python3 -c "import json; r=json.loads(open('$O/aw_b.json').read().strip().splitlines()[-1]); print(json.dumps({'rep': $rep, 'value': r['value'], 'ms_per_step': r['ms_per_step'], 'verified': r['verified']}))" >> $O/aw_spread.jsonl
done
echo "exit 0"
