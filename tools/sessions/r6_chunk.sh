#!/bin/bash
# Round 6: multi-step block sums of C steps at once (MIINT_MS_CHUNK) against one per step;
# the 1/8 share's work and N = 1e9, 20-step batches, alternating builds.
set -o pipefail
O=gpurun_out/chunk; mkdir -p $O
B="build/bin build/ab_c2/bin build/ab_c4/bin"
bash tools/variant_ab.sh $O/s8.jsonl "miint bench --n 1.25e8 --slots 20" $B > /dev/null &&
bash tools/variant_ab.sh $O/s4.jsonl "miint bench --n 2.5e8 --slots 20" $B > /dev/null &&
bash tools/variant_ab.sh $O/g1.jsonl "miint bench --n 1e9 --slots 20" $B > /dev/null
rc=$?; echo "rc=$rc"; exit $rc
