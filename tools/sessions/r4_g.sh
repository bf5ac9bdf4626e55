# round 4 session G: buffer-load staging at HEAD — the 2-D tests, the 2-D rows, then the
# whole GPU suite and the bench at HEAD
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py tests/test_lds_poison_gpu.py -k "table2d or poison" \
  > gpurun_out/r4/gputests_g1.txt 2>&1
rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/r4/gputests_g1.txt; exit $rc; }
grep -E "FAILED|^E " gpurun_out/r4/gputests_g1.txt | cut -c1-300 || true
tail -2 gpurun_out/r4/gputests_g1.txt
[ $rc -eq 0 ] || exit 1
out=gpurun_out/r4/t2d_bufload.jsonl; : > $out
for rep in 1 2 3; do for sl in full 0/2 0/4 0/8; do
  extra=(); [ "$sl" != full ] && extra=(--slice "$sl")
  line=$(timeout -k 10 60 build/bin/miint table2d --grid 4096 --iters 640 "${extra[@]}" | grep '^{' | tail -1) || exit 1
  echo "{\"rep\": $rep, \"slice_arg\": \"$sl\", ${line#\{}" >> $out
done; done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$out'):
    r=json.loads(l); d[(r['slice_arg'],r['phases'])].append(round(r['ms_per_integration']*1e3,3))
for k in sorted(d): print(k,d[k])"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  > gpurun_out/r4/gputests_full_g.txt 2>&1
rc=$?
tail -3 gpurun_out/r4/gputests_full_g.txt
grep -E "FAILED|^E " gpurun_out/r4/gputests_full_g.txt | cut -c1-300 | head -30 || true
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_g.json 2> gpurun_out/r4/bench_g.log || { tail -20 gpurun_out/r4/bench_g.log; exit 1; }
cut -c1-300 gpurun_out/r4/bench_g.json
