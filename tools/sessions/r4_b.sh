# round 4 session B: 2-D phases on slices (explicit 1-4), slice shapes, settled one-shot,
# bench at HEAD, full GPU tests
set -uo pipefail
mkdir -p gpurun_out/r4
tag() { python3 -c 'import json,sys
extra = json.loads(sys.argv[1])
for l in sys.stdin:
    if l.startswith("{"):
        r = json.loads(l); r.update(extra); print(json.dumps(r))' "$1"; }
: > gpurun_out/r4/t2d_phases_explicit.jsonl
for rep in 1 2; do
  for sl in 0/8 0/4 0/2 full; do
    for ph in 1 2 3 4; do
      extra=(); [ "$sl" != full ] && extra=(--slice "$sl")
      timeout -k 10 90 build/bin/miint table2d --grid 4096 --iters 320 --phases $ph "${extra[@]}" | tag "{\"slice_arg\": \"$sl\", \"phases_arg\": $ph, \"rep\": $rep}" >> gpurun_out/r4/t2d_phases_explicit.jsonl || exit 1
    done
  done
done
: > gpurun_out/r4/t2d_slice_shapes.jsonl
for rep in 1 2; do
  for mw in 0 256 128; do
    for sl in 0/8 0/4; do
      for ph in 0 4; do
        timeout -k 10 90 build/bin/miint table2d --grid 4096 --iters 320 --slice $sl --min-wg $mw --phases $ph | tag "{\"slice_arg\": \"$sl\", \"min_wg_arg\": $mw, \"phases_arg\": $ph, \"rep\": $rep}" >> gpurun_out/r4/t2d_slice_shapes.jsonl || exit 1
      done
    done
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/r4/t2d_phases_explicit.jsonl"):
    r = json.loads(l); d[(r["slice_arg"], r["phases_arg"])].append(r["ms_per_integration"] * 1e3)
for k in sorted(d): print("phases", k, [round(x, 3) for x in d[k]])
d = collections.defaultdict(list)
for l in open("gpurun_out/r4/t2d_slice_shapes.jsonl"):
    r = json.loads(l); d[(r["slice_arg"], r["min_wg_arg"], r["phases_arg"], r["phases"])].append(r["ms_per_integration"] * 1e3)
for k in sorted(d): print("shape", k, [round(x, 3) for x in d[k]])
PY
timeout -k 10 120 python tools/one_shot_probe.py 50 > gpurun_out/r4/one_shot_probe_settled.jsonl 2>/dev/null || exit 1
cut -c1-220 gpurun_out/r4/one_shot_probe_settled.jsonl
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_b.json 2> gpurun_out/r4/bench_b.log || exit 1
python3 -c '
import json
r = json.load(open("gpurun_out/r4/bench_b.json"))
print("bench", r["value"], r["verified"], r["single_shot_1e9"]["ms_one_shot"], r["single_shot_1e9"]["best_form"], r["baseline4_fp32"]["value"], r["baseline5_table2d_4096"]["ms_per_integration"], r.get("series_exact_div", {}).get("value"))
'
timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r4/gputests_full.txt 2>&1; tail -5 gpurun_out/r4/gputests_full.txt
