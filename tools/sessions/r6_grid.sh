#!/bin/bash
# Round 6: multi-step grid at the 1/8 and 1/4 shares (rotation balances a partial tile round
# over the batch), interleaved, 20-step batches with the 1-rank RCCL stage.
set -o pipefail
O=gpurun_out/grid; mkdir -p $O
timeout -k 10 240 python -u tools/batch_ab.py --slice 8 --steps 20 --slots 20 --collective \
  --values-may-differ --variant grid=256 --variant grid=512 --variant grid=768 \
  --variant grid=1024 --jsonl $O/s8.jsonl > $O/s8.log 2>&1 &&
timeout -k 10 240 python -u tools/batch_ab.py --slice 4 --steps 20 --slots 20 --collective \
  --values-may-differ --variant grid=512 --variant grid=1024 --variant grid=1536 \
  --jsonl $O/s4.jsonl > $O/s4.log 2>&1
rc=$?; echo "rc=$rc"; tail -8 $O/s8.log; tail -6 $O/s4.log; exit $rc
