#!/bin/bash
# r5 session AE: wave-state counters of the multi-step kernel, N = 1e9 vs the 1/8 share
set -o pipefail
cd "$GRAFT_REPO_ROOT"
REPO=$(pwd)
O=$REPO/gpurun_out/r5/ae_pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
C2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
for n in 1e9 1.25e8; do
  it=960; [ "$n" = "1.25e8" ] && it=7680
  timeout -s KILL 90 rocprofv3 --pmc $C1 --kernel-trace --output-format csv -d $O/n${n}_c1 -o run -- \
    $REPO/build/bin/miint bench --n $n --slots 48 --iters $it > $O/n${n}_c1.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $C2 --kernel-trace --output-format csv -d $O/n${n}_c2 -o run -- \
    $REPO/build/bin/miint bench --n $n --slots 48 --iters $it > $O/n${n}_c2.log 2>&1 || exit 1
done
echo "exit 0"
