#!/bin/bash
# r5 session AP: clock and VALU issue of the multi-step kernel on the 1/8 share in 64-step
# dispatches (>= 500 us, long enough for the GRBM clock reading) against N = 1e9
set -o pipefail
cd "$GRAFT_REPO_ROOT"
R=$PWD
O=$R/gpurun_out/r5/pmc_ap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
timeout -k 10 120 rocprofv3 --pmc $G1 --kernel-trace --output-format csv -d $O/pi4_series_exact_share8_G1 -o run -- "$R/build/bin/miint" bench --n 1.25e8 --slots 64 --iters 3840 > $O/s8.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc $G1 --kernel-trace --output-format csv -d $O/pi4_series_exact_G1 -o run -- "$R/build/bin/miint" bench --slots 64 --iters 512 > $O/g1.log 2>&1
echo "exit $?"
