#!/bin/bash
# r5 session K: multi-step grid at the strong shares of N = 1e9 (20-step batches), series_exact
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
: > $O/k_grid.jsonl
for rep in 1 2; do
  for n in 5e8 2.5e8 1.25e8; do
    for g in 0 256 512 768 1024 1280 1536 1792; do
      line=$(timeout -k 10 60 build/bin/miint bench --integrand pi4 --n $n --iters 400 --slots 20 --grid $g | grep '^{' | tail -1) || exit 1
      echo "{\"rep\": $rep, \"grid_req\": $g, ${line#\{}" >> $O/k_grid.jsonl
    done
  done
done
echo "exit 0"
