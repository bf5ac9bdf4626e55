# round 4 session D: whole-row staging (one lane offset) at HEAD — the 2-D tests incl. LDS
# poison — then the 2-D kernel variant A/B (tile height 30 = 5 workgroups per CU, full-tile
# prefetch) at 4 and 8 step phases
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py tests/test_lds_poison_gpu.py -k "table2d or poison" \
  > gpurun_out/r4/gputests_d.txt 2>&1
rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/r4/gputests_d.txt; exit $rc; }
grep -E "FAILED|^E " gpurun_out/r4/gputests_d.txt | cut -c1-300 || true
tail -2 gpurun_out/r4/gputests_d.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 700 bash tools/t2d_variant_ab.sh gpurun_out/r4/t2d_variant_ab.jsonl \
  build/ab_base/bin build/ab_sh30/bin build/ab_pf/bin build/ab_sh30pf/bin || exit 1
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r4/t2d_variant_ab.jsonl")]
d = collections.defaultdict(list)
val = collections.defaultdict(set)
for r in rows:
    k = (r["slice_arg"] or "full", r["phases_arg"], r["build"].split("/")[1])
    d[k].append(round(r["ms_per_integration"] * 1e3, 3))
    val[(r["slice_arg"], r["phases_arg"])].add(r.get("result", r.get("partial")))
for k in sorted(d):
    print(k, d[k])
print("distinct values per (slice, phases):", {k: len(v) for k, v in val.items()})
PY
