# round 4 session S: 1-step batches of chained plans as the fused launch — the bitwise /
# batch / one-shot GPU tests, the settled one-shot probe and a bench
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py tests/test_loopback_gpu.py > gpurun_out/r4/gputests_s.txt 2>&1
rc=$?
tail -2 gpurun_out/r4/gputests_s.txt
grep -E "FAILED|^E " gpurun_out/r4/gputests_s.txt | cut -c1-300 | head -20 || true
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/one_shot_probe.py 60 > gpurun_out/r4/one_shot_probe_s.jsonl 2>/dev/null || exit 1
cut -c1-200 gpurun_out/r4/one_shot_probe_s.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_s20.json 2> gpurun_out/r4/bench_s20.log || { tail -20 gpurun_out/r4/bench_s20.log; exit 1; }
python3 -c "
import json
r=json.loads(open('gpurun_out/r4/bench_s20.json').read().strip().splitlines()[-1])
print(r['value'], r['verified'], r['single_shot_1e9']['best_form'], r['single_shot_1e9']['ms_one_shot'], {k: round(v['median_us'],2) for k, v in r['single_shot_1e9']['forms'].items()})"
