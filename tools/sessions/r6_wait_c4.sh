#!/bin/bash
# Round 6: the wait counters (profile_counters.sh G5) at the 1/8 share for the chunked block
# sum (MIINT_MS_CHUNK=4 build: a barrier every 4 steps) next to the default build.
set -o pipefail
R=$(pwd); O=$R/gpurun_out/pmc_c4; mkdir -p $O
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU GRBM_GUI_ACTIVE"
cd /tmp && export TMPDIR=/tmp
for b in bin ab_c4/bin; do
  t=$(echo $b | tr '/' '_')
  timeout -k 10 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/share8_$t -o run -- \
    $R/build/$b/miint bench --n 1.25e8 --slots 20 --iters 2000 --settle 2000 > $O/share8_$t.log 2>&1 || exit 1
done
cd $R && python3 tools/summarize_counters.py $O > gpurun_out/pmc_c4.md
rc=$?; echo "rc=$rc"; cat gpurun_out/pmc_c4.md; exit $rc
