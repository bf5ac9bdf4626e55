# round 4 session J: per-batch fixed cost of the headline's timed region (graph vs direct)
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 180 python tools/replay_overhead_probe.py > gpurun_out/r4/replay_overhead.jsonl 2> gpurun_out/r4/replay_overhead.log || { tail -5 gpurun_out/r4/replay_overhead.log; exit 1; }
cat gpurun_out/r4/replay_overhead.jsonl
