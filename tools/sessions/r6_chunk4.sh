#!/bin/bash
# Round 6: 4-step block sums as the Pi4 default (build/bin) against the round-5 kernel
# (build/ab_c1: MIINT_MS_CHUNK=1) — the driver's shape at G = 1 and the shares, alternating
# builds — then the GPU suite and the default bench at the new default.
set -o pipefail
O=gpurun_out/chunk4; mkdir -p $O
B="build/bin build/ab_c1/bin"
bash tools/variant_ab.sh $O/s8.jsonl "miint bench --n 1.25e8 --slots 20" $B > /dev/null &&
bash tools/variant_ab.sh $O/s4.jsonl "miint bench --n 2.5e8 --slots 20" $B > /dev/null &&
bash tools/variant_ab.sh $O/g1.jsonl "miint bench --n 1e9 --slots 20" $B > /dev/null &&
bash tools/variant_ab.sh $O/s8b.jsonl "miint bench --n 1.25e8 --slots 20" $B > /dev/null &&
bash tools/variant_ab.sh $O/g1b.jsonl "miint bench --n 1e9 --slots 20" $B > /dev/null &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/gputests.txt 2>&1 &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err
rc=$?; echo "rc=$rc"; tail -2 $O/gputests.txt; head -c 400 $O/bench20.json; exit $rc
