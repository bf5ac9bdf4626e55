# round 4 session O: the multi-rank bench WITH every extra (the driver's 8-GPU record runs
# them all), two and four RCCL ranks sharing the GPU, and the driver's torchrun form
set -uo pipefail
mkdir -p gpurun_out/r4
export MIINT_OVERSUBSCRIBE=1
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/r4/bench_np2_extras.json 2> gpurun_out/r4/bench_np2_extras.log || { tail -20 gpurun_out/r4/bench_np2_extras.log; exit 1; }
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/r4/bench_np2_extras.json").read().strip().splitlines()[-1])
print("np2 verified", r["verified"], r.get("extras_error"), r["value"], r.get("rccl_transport"), r.get("transport_error"))
for k, v in r.items():
    if isinstance(v, dict) and "verified" in v:
        print(" ", k, v["verified"])
PY
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29733 bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/r4/bench_np4_extras.json 2> gpurun_out/r4/bench_np4_extras.log || { tail -20 gpurun_out/r4/bench_np4_extras.log; exit 1; }
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/r4/bench_np4_extras.json").read().strip().splitlines()[-1])
print("np4 verified", r["verified"], r.get("extras_error"), r["value"], r.get("rccl_transport"), r.get("launcher"))
for k, v in r.items():
    if isinstance(v, dict) and "verified" in v:
        print(" ", k, v["verified"])
PY
