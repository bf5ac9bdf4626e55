# round 4 session Q: multi-step replays past residency by default — the 2-D GPU tests
# (incl. 8192^2 bitwise vs chained, loopback ranks, poison) and the 8192^2 / 6144^2 rows
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py tests/test_lds_poison_gpu.py tests/test_loopback_gpu.py \
  tests/test_gpu_shared_rccl.py -k "table2d or poison" > gpurun_out/r4/gputests_q.txt 2>&1
rc=$?
tail -2 gpurun_out/r4/gputests_q.txt
grep -E "FAILED|^E " gpurun_out/r4/gputests_q.txt | cut -c1-300 | head -20 || true
[ $rc -eq 0 ] || exit $rc
for g in 8192 6144 4096; do
  timeout -k 10 60 build/bin/miint table2d --grid $g --iters 640 | cut -c1-330
done
