#!/usr/bin/env bash
# Multi-rank RCCL on ONE GPU (MIINT_OVERSUBSCRIBE=1, comm.hpp ranks_share_devices): W ranks,
# one process each, share device 0; each names itself a host of its own (NCCL_HOSTID) and
# RCCL joins them over its socket transport on loopback. Runs every native CLI and bench.py
# (native and torch data planes) with real RCCL communicators of world 2 and 4. Each step
# under its own limit; stops at the first failure. Output: gpurun_out/shared_rccl/.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/shared_rccl
mkdir -p "$out"
export MIINT_OVERSUBSCRIBE=1 NCCL_DEBUG=INFO NCCL_DEBUG_SUBSYS=INIT,NET
step() {  # step NAME LIMIT CMD...: stdout -> NAME.json(l), stderr -> NAME.log
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "$out/$name.out" 2> "$out/$name.log"
  grep '^{' "$out/$name.out" || tail -3 "$out/$name.out"
}
run=build/bin/miintrun
step riemann_np2 120 $run -np 2 -- build/bin/riemann --integrand pi4 --iters 20 --json
step riemann_sin_np4 120 $run -np 4 -- build/bin/riemann --iters 5 --json
step trainscan_np2 120 $run -np 2 -- build/bin/trainscan --iters 3 --json
step cintegrate_np2 120 $run -np 2 -- build/bin/cintegrate --iters 3 --json
step miint_bench_np2 120 $run -np 2 -- build/bin/miint bench --integrand pi4 --iters 20
step miint_table2d_np2 120 $run -np 2 -- build/bin/miint table2d --grid 4096
step bench_native_np2 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-extras
step bench_torch_np2 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-extras --comm torch
step bench_native_np4 300 python bench.py --gpus 4 --steps 20 --warmup 5 --no-extras
step bench_strong_np2 300 python bench.py --gpus 2 --steps 20 --warmup 5 --no-extras --scaling strong
# RCCL prints its INFO lines on stdout: transport and topology of every communicator
for f in "$out"/*.out; do
  echo "== $(basename "$f" .out)"
  grep -o 'nRanks [0-9]* nNodes [0-9]* localRanks [0-9]*\|via NET/Socket/[0-9]*\|Using \[0\]lo:[0-9.]*\|Init COMPLETE' "$f" | sort | uniq -c || true
done > "$out/nccl_summary.txt"
echo done
