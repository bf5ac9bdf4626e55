# round 4 session C: PMC roofline at HEAD, settled one-shot (event-free host timing),
# shared-GPU RCCL at HEAD
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 120 python tools/one_shot_probe.py 50 > gpurun_out/r4/one_shot_probe_c.jsonl 2>/dev/null || exit 1
cut -c1-220 gpurun_out/r4/one_shot_probe_c.jsonl
bash tools/sessions/r4_pmc.sh > gpurun_out/r4/pmc_session.txt 2>&1 || { tail -20 gpurun_out/r4/pmc_session.txt; exit 1; }
tail -30 gpurun_out/r4/roofline.md
timeout -k 10 600 bash tools/shared_gpu_rccl.sh > gpurun_out/r4/shared_rccl_c.txt 2>&1; tail -40 gpurun_out/shared_rccl/summary.md
