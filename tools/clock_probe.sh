#!/usr/bin/env bash
# Sustained shader clock under each hot kernel: run `miint bench` for ~2 s per workload in the
# background and sample the current SCLK with rocm-smi / amd-smi while it runs. The roofline
# (tools/roofline.py) prices VALU issue at the 2.4 GHz peak; this measures what the clock
# actually is under a saturating fp64 / fp32 VALU load. Output: gpurun_out/clock_probe.txt
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/clock_probe.txt
mkdir -p gpurun_out
: > "$out"
probe() {  # probe NAME ITERS ARGS...
  local name=$1 iters=$2; shift 2
  timeout -k 10 60 build/bin/miint bench --iters "$iters" "$@" > "gpurun_out/clock_$name.json" 2>&1 &
  local pid=$!
  sleep 0.8
  for i in 1 2 3 4 5 6; do
    if ! kill -0 $pid 2>/dev/null; then break; fi
    echo "$name sample$i $(rocm-smi --showclocks 2>/dev/null | grep -i 'sclk' | head -1)" >> "$out"
    sleep 0.2
  done
  wait $pid || { echo "$name bench failed" >> "$out"; return 1; }
  echo "$name $(grep '^{' "gpurun_out/clock_$name.json" | tail -1)" >> "$out"
}
echo "idle $(rocm-smi --showclocks 2>/dev/null | grep -i 'sclk' | head -1)" >> "$out"
if [ "${SHARES:-0}" = 1 ]; then
  # the headline's per-GPU shares of a G-GPU strong-scaled step, in the driver's 20-step
  # batches (profiles/r6/batch_tail.md: does the share run at G = 1's clock?)
  probe share1 30000 --integrand pi4 --slots 20 && \
  probe share8 200000 --integrand pi4 --n 1.25e8 --slots 20 && \
  probe share4 110000 --integrand pi4 --n 2.5e8 --slots 20 && \
  probe share8_again 200000 --integrand pi4 --n 1.25e8 --slots 20 && \
  probe share1_again 30000 --integrand pi4 --slots 20
else
  probe pi4_series 30000 --integrand pi4 && \
  probe pi4_fp32 50000 --integrand pi4 --dtype fp32 && \
  probe sin_series 25000 --integrand sin && \
  probe pi4_ieee 6000 --integrand pi4 --div ieee
fi
rocm-smi --showclocks >> "$out" 2>&1 || true
echo done
