# round 4 session K: final validation at HEAD — smoke, the whole GPU suite, the bench in the
# driver's shape and at 400 steps, a kernel-trace profile of the driver-shape bench, and the
# 2-D PMC rows with buffer-load staging
set -uo pipefail
mkdir -p gpurun_out/r4
R=$(pwd)
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4/smoke_k.txt 2>&1 || { tail -20 gpurun_out/r4/smoke_k.txt; exit 1; }
tail -1 gpurun_out/r4/smoke_k.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r4/gputests_full_k.txt 2>&1
rc=$?
tail -2 gpurun_out/r4/gputests_full_k.txt
grep -E "FAILED|^E " gpurun_out/r4/gputests_full_k.txt | cut -c1-300 | head -30 || true
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_k20.json 2> gpurun_out/r4/bench_k20.log || { tail -20 gpurun_out/r4/bench_k20.log; exit 1; }
cut -c1-300 gpurun_out/r4/bench_k20.json
timeout -k 10 300 python bench.py > gpurun_out/r4/bench_k400.json 2> gpurun_out/r4/bench_k400.log || { tail -20 gpurun_out/r4/bench_k400.log; exit 1; }
cut -c1-300 gpurun_out/r4/bench_k400.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r4/prof_k" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-extras > "$R/gpurun_out/r4/prof_k.log" 2>&1 || { tail -20 "$R/gpurun_out/r4/prof_k.log"; exit 1; }
cd "$R"
find gpurun_out/r4/prof_k -name "*kernel_stats.csv" | head -3
rm -rf gpurun_out/pmc
ONLY="table2d table2d_slice8" timeout -k 10 400 bash tools/profile_counters.sh > gpurun_out/r4/pmc_k.log 2>&1 || { tail -20 gpurun_out/r4/pmc_k.log; exit 1; }
python3 tools/roofline.py gpurun_out/pmc > gpurun_out/r4/roofline_t2d_k.md
cat gpurun_out/r4/roofline_t2d_k.md
