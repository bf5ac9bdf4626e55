#!/usr/bin/env bash
# PMC counters (VALU instructions per sample) of the fp32 and fp64 sin / table / train / poly
# kernels, one counter group per run (--pmc with --kernel-trace only).
#   tools/fp32_pmc.sh ; python tools/summarize_counters.py gpurun_out/pmc32 > profiles/r2/fp32_counters.md
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
REPO=$(pwd)
OUT=$REPO/gpurun_out/pmc32
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE"
run() {  # name, counters, command...
  local name=$1 ctrs=$2; shift 2
  timeout -k 10 120 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv \
    -d "$OUT/${name}_G1" -o run -- "$@" > "$OUT/${name}_G1.log" 2>&1
}
for f in sin table train poly; do
  run ${f}_fp32 "$G1" "$REPO/build/bin/miint" bench --iters 10 --integrand $f --dtype fp32
  run ${f}_fp64 "$G1" "$REPO/build/bin/miint" bench --iters 10 --integrand $f
done
echo "pmc32 done"
