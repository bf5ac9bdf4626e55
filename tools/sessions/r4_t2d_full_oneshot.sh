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
timeout -k 10 300 bash tools/variant_ab.sh gpurun_out/r4/t2d_pf_ab_full.jsonl "miint table2d --grid 4096 --iters 320" build/bin build/ab_t2dpf/bin > /dev/null || exit 1
timeout -k 10 300 bash tools/variant_ab.sh gpurun_out/r4/t2d_pf_ab_slice8.jsonl "miint table2d --grid 4096 --iters 320 --slice 0/8" build/bin build/ab_t2dpf/bin > /dev/null || exit 1
python3 -c '
import json
for f in ("gpurun_out/r4/t2d_pf_ab_full.jsonl", "gpurun_out/r4/t2d_pf_ab_slice8.jsonl"):
    for l in open(f):
        r=json.loads(l); print(f[-12:], r["build"], r["ms_per_integration"], r.get("phases"), r.get("partial", r.get("rel_err_vs_oracle")))
'
: > gpurun_out/r4/t2d_slice_shapes.jsonl
for rep in 1 2; do
  for mw in 0 256 128; do
    for sl in 0/8 0/4 0/2; do
      timeout -k 10 90 build/bin/miint table2d --grid 4096 --iters 320 --slice $sl --min-wg $mw | sed "s/^{/{\"min_wg_arg\": $mw, \"slice_arg\": \"$sl\", /" >> gpurun_out/r4/t2d_slice_shapes.jsonl || exit 1
    done
  done
done
python3 -c '
import json
for l in open("gpurun_out/r4/t2d_slice_shapes.jsonl"):
    r=json.loads(l); print(r["slice_arg"], r["min_wg_arg"], r["phases"], r["resident_per_cu"], r["ms_per_integration"])
'
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_b.json 2> gpurun_out/r4/bench_b.log || exit 1
python3 -c '
import json
r = json.load(open("gpurun_out/r4/bench_b.json"))
print("bench", r["value"], r["verified"], r["single_shot_1e9"]["ms_one_shot"], r["baseline4_fp32"]["value"], r["baseline5_table2d_4096"]["ms_per_integration"], r.get("series_exact_div", {}).get("value"))
'
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r4/gputests_full.txt 2>&1; tail -5 gpurun_out/r4/gputests_full.txt
