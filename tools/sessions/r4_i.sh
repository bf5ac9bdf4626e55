# round 4 session I: 2-D row-change A/B — fresh lines at every change (no carried next line,
# 58 VGPRs) with and without the full-tile prefetch, against HEAD — at 16 phases
set -uo pipefail
mkdir -p gpurun_out/r4
PHASES="16" timeout -k 10 600 bash tools/t2d_variant_ab.sh gpurun_out/r4/t2d_fresh_ab.jsonl \
  build/ab_base/bin build/ab_fresh/bin build/ab_freshpf/bin || exit 1
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r4/t2d_fresh_ab.jsonl")]
d = collections.defaultdict(list)
val = collections.defaultdict(set)
for r in rows:
    d[(r["slice_arg"] or "full", r["build"].split("/")[1])].append(round(r["ms_per_integration"] * 1e3, 3))
    val[r["slice_arg"]].add(r.get("result", r.get("partial")))
for k in sorted(d):
    print(k, d[k])
print("distinct values per slice:", {k: len(v) for k, v in val.items()})
PY
