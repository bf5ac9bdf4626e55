# round 4 session E: 30-row tiles + 8 auto phases at HEAD — the 2-D tests — then the shape
# sweep (rows per wave x phases 8 / 16) on the default build
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py tests/test_lds_poison_gpu.py -k "table2d or poison" \
  > gpurun_out/r4/gputests_e.txt 2>&1
rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/r4/gputests_e.txt; exit $rc; }
grep -E "FAILED|^E " gpurun_out/r4/gputests_e.txt | cut -c1-300 || true
tail -2 gpurun_out/r4/gputests_e.txt
[ $rc -eq 0 ] || exit 1
timeout -k 10 800 bash tools/t2d_shape_sweep.sh gpurun_out/r4/t2d_shape_sweep.jsonl build/bin 8 16 || exit 1
python3 - <<'PY'
import json, collections
rows = [json.loads(l) for l in open("gpurun_out/r4/t2d_shape_sweep.jsonl")]
d = collections.defaultdict(list)
for r in rows:
    d[(r["slice_arg"], r["workgroups"], r["phases"], r["resident_per_cu"])].append(round(r["ms_per_integration"] * 1e3, 3))
for k in sorted(d):
    print(k, d[k])
PY
