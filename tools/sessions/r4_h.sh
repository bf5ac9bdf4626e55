# round 4 session H: --force-collective bench (single_shot through the collective plan), then
# the shared-GPU RCCL sweep at HEAD
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread \
  tests/test_gpu_runtime.py -k "force_collective or bench_contract" > gpurun_out/r4/gputests_h.txt 2>&1
rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/r4/gputests_h.txt; exit $rc; }
grep -E "FAILED|^E " gpurun_out/r4/gputests_h.txt | cut -c1-300 || true
tail -2 gpurun_out/r4/gputests_h.txt
timeout -k 10 700 bash tools/shared_gpu_rccl.sh > gpurun_out/r4/shared_rccl_h.txt 2>&1
rc=$?
tail -5 gpurun_out/r4/shared_rccl_h.txt
[ $rc -eq 0 ] || exit $rc
tail -40 gpurun_out/shared_rccl/summary.md
