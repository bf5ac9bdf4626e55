#!/bin/bash
# r5 session S: multi-step launch duration against its step count K (kernel trace), at the
# 1/8 share (N = 1.25e8) and at N = 1e9: fit duration = K c + F to size the per-launch cost F
set -o pipefail
cd "$GRAFT_REPO_ROOT"
REPO=$(pwd)
O=$REPO/gpurun_out/r5/s_fit2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for n in 1.25e8 1e9; do
  for k in 1 2 4 8 16 32 64; do
    it=$((k * 16)); st=6000; [ "$n" = "1e9" ] && it=$((k * 8)) && st=800
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n${n}_k$k -o run -- \
      $REPO/build/bin/miint bench --n $n --slots $k --iters $it > $O/n${n}_k$k.log 2>&1 || exit 1
  done
done
echo "exit 0"
