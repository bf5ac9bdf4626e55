# 2-D full-field phases past the occupancy API's residency, device info, one-shot kernel trace
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 60 build/bin/miint info > gpurun_out/r4/miint_info.txt 2>&1 || exit 1
: > gpurun_out/r4/t2d_full_phases.jsonl
for rep in 1 2; do
  for ph in 1 2 3 4; do
    timeout -k 10 90 build/bin/miint table2d --grid 4096 --iters 320 --phases $ph >> gpurun_out/r4/t2d_full_phases.jsonl || exit 1
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_oneshot" -o oneshot --output-format csv -- python3 tools/one_shot_probe.py 30 > gpurun_out/r4/oneshot_prof.log 2>&1 || exit 1
cat gpurun_out/r4/miint_info.txt
python3 -c '
import json
for l in open("gpurun_out/r4/t2d_full_phases.jsonl"):
    r=json.loads(l); print(r["phases"], r["resident_per_cu"], r["ms_per_integration"], r["rel_err_vs_oracle"])
'
find gpurun_out/prof_oneshot -name "*.csv" | head
timeout -k 10 300 bash tools/variant_ab.sh gpurun_out/r4/fused_tail_ab.jsonl "riemann --integrand pi4 --json --iters 20 --no-multistep" build/bin build/ab_tail/bin > /dev/null || exit 1
python3 -c '
import json
for l in open("gpurun_out/r4/fused_tail_ab.jsonl"):
    r=json.loads(l); print(r["build"], r["ms_one_shot"], r["device_ms"], r["grid"], r["result"])
'
