# round 4 session R: the last HEAD (after multi-step past residency) — smoke, the whole GPU suite, the bench (driver shape)
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4/smoke_r.txt 2>&1 || { tail -20 gpurun_out/r4/smoke_r.txt; exit 1; }
tail -1 gpurun_out/r4/smoke_r.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r4/gputests_full_r.txt 2>&1
rc=$?
tail -2 gpurun_out/r4/gputests_full_r.txt
grep -E "FAILED|^E " gpurun_out/r4/gputests_full_r.txt | cut -c1-300 | head -30 || true
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_r20.json 2> gpurun_out/r4/bench_r20.log || { tail -20 gpurun_out/r4/bench_r20.log; exit 1; }
cut -c1-300 gpurun_out/r4/bench_r20.json
timeout -k 10 120 build/bin/riemann --integrand pi4 --n 1e9 --iters 20 --json | cut -c1-600
