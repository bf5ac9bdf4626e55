# round 4 session T: the last HEAD (after 1-step fused batches) — smoke, the whole GPU suite, the bench (driver shape)
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r4/smoke_t.txt 2>&1 || { tail -20 gpurun_out/r4/smoke_t.txt; exit 1; }
tail -1 gpurun_out/r4/smoke_t.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/r4/gputests_full_t.txt 2>&1
rc=$?
tail -2 gpurun_out/r4/gputests_full_t.txt
grep -E "FAILED|^E " gpurun_out/r4/gputests_full_t.txt | cut -c1-300 | head -30 || true
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r4/bench_t20.json 2> gpurun_out/r4/bench_t20.log || { tail -20 gpurun_out/r4/bench_t20.log; exit 1; }
cut -c1-300 gpurun_out/r4/bench_t20.json
timeout -k 10 120 build/bin/riemann --integrand pi4 --n 1e9 --iters 20 --json | cut -c1-600
