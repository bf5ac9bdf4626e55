#!/usr/bin/env bash
# Multi-rank RCCL on ONE GPU (MIINT_OVERSUBSCRIBE=1, comm.hpp ranks_share_devices): W ranks,
# one process each, share device 0; each names itself a host of its own (NCCL_HOSTID) and
# RCCL joins them over its socket transport on loopback. Runs every native CLI and bench.py
# (native and torch data planes) with real RCCL communicators of world 2 and 4, next to the
# same tool on one rank: every tool now starts its ranks' clocks behind a collective barrier
# and reports the slowest rank's time, so no multi-rank record on the one GPU may beat the
# single-rank one. Each step under its own limit; stops at the first failure.
# Output: gpurun_out/shared_rccl/ (records.jsonl: one record per step, tagged).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/shared_rccl
mkdir -p "$out"
rm -f "$out/records.jsonl"
step() {  # step NAME LIMIT CMD...: stdout -> NAME.out, stderr -> NAME.log, records tagged
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "$out/$name.out" 2> "$out/$name.log"
  grep '^{' "$out/$name.out" | python3 -c '
import json, sys
for l in sys.stdin:
    r = json.loads(l); r["step"] = sys.argv[1]; print(json.dumps(r))' "$name" | tee -a "$out/records.jsonl"
}
run=build/bin/miintrun
pi=(--integrand pi4 --n 1e9 --iters 20 --json)
step riemann_np1 120 build/bin/riemann "${pi[@]}"
step riemann_np2 120 env MIINT_OVERSUBSCRIBE=1 $run -np 2 -- build/bin/riemann "${pi[@]}"
step riemann_np4 120 env MIINT_OVERSUBSCRIBE=1 $run -np 4 -- build/bin/riemann "${pi[@]}"
step riemann_sin_np1 120 build/bin/riemann --iters 5 --json
step riemann_sin_np4 120 env MIINT_OVERSUBSCRIBE=1 $run -np 4 -- build/bin/riemann --iters 5 --json
step riemann_parity_np3 120 env MIINT_OVERSUBSCRIBE=1 $run -np 3 -- build/bin/riemann --parity --json
step riemann_parity_np8 120 env MIINT_OVERSUBSCRIBE=1 $run -np 8 -- build/bin/riemann --parity --json
step trainscan_np1 120 build/bin/trainscan --iters 3 --json
step trainscan_np2 120 env MIINT_OVERSUBSCRIBE=1 $run -np 2 -- build/bin/trainscan --iters 3 --json
step cintegrate_np1 120 build/bin/cintegrate --json
step cintegrate_np2 120 env MIINT_OVERSUBSCRIBE=1 $run -np 2 -- build/bin/cintegrate --json
step miint_bench_np1 120 build/bin/miint bench --integrand pi4 --iters 20
step miint_bench_np2 120 env MIINT_OVERSUBSCRIBE=1 $run -np 2 -- build/bin/miint bench --integrand pi4 --iters 20
step miint_table2d_np1 120 build/bin/miint table2d --grid 4096
step miint_table2d_np2 120 env MIINT_OVERSUBSCRIBE=1 $run -np 2 -- build/bin/miint table2d --grid 4096
step miint_comm_np2 120 env MIINT_OVERSUBSCRIBE=1 $run -np 2 -- build/bin/miint comm --max-bytes 1e6 --iters 5
step bench_native_np1 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extras
step bench_native_np2 300 env MIINT_OVERSUBSCRIBE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-extras
step bench_torch_np2 300 env MIINT_OVERSUBSCRIBE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-extras --comm torch
step bench_native_np4 300 env MIINT_OVERSUBSCRIBE=1 python bench.py --gpus 4 --steps 20 --warmup 5 --no-extras
step bench_strong_np2 300 env MIINT_OVERSUBSCRIBE=1 python bench.py --gpus 2 --steps 20 --warmup 5 --no-extras --scaling strong
python3 tools/shared_rccl_report.py "$out/records.jsonl" > "$out/summary.md" || echo "WARNING: a multi-rank record beats its one-rank rate"
cat "$out/summary.md"
echo done
