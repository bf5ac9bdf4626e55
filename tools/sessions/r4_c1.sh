# round 4 session C1: the changed paths at HEAD (2-D auto shape/phases, 1-step batches as the
# fused launch, series_exact bound), the settled one-shot probe, the 2-D CLI auto rows, bench
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py -k "table2d or multistep or series_exact or one_shot" \
  > gpurun_out/r4/gputests_c1.txt 2>&1
rc=$?
# an assertion (1) does not stop the session; a crash, abort or time limit does
[ $rc -le 1 ] || { tail -40 gpurun_out/r4/gputests_c1.txt; exit $rc; }
grep -E "FAILED|^E " gpurun_out/r4/gputests_c1.txt | cut -c1-300 || true
tail -3 gpurun_out/r4/gputests_c1.txt
timeout -k 10 120 python tools/one_shot_probe.py 50 > gpurun_out/r4/one_shot_probe_c.jsonl 2>/dev/null || exit 1
cut -c1-200 gpurun_out/r4/one_shot_probe_c.jsonl
: > gpurun_out/r4/t2d_auto_c.jsonl
for sl in 0/1 0/2 0/4 0/8; do
  for rep in 1 2; do
    timeout -k 10 60 build/bin/miint table2d --grid 4096 --iters 640 --slice "$sl" >> gpurun_out/r4/t2d_auto_c.jsonl || exit 1
  done
done
cut -c1-260 gpurun_out/r4/t2d_auto_c.jsonl
timeout -k 10 300 python bench.py > gpurun_out/r4/bench_c1.json 2> gpurun_out/r4/bench_c1.log || { tail -20 gpurun_out/r4/bench_c1.log; exit 1; }
cut -c1-400 gpurun_out/r4/bench_c1.json
