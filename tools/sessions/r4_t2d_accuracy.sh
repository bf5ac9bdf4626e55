mkdir -p gpurun_out/r4 && timeout -k 10 400 bash tools/table2d_phases_ab.sh > gpurun_out/r4/t2d_ab.txt 2>&1 && timeout -k 10 300 python tools/accuracy_ab.py > gpurun_out/r4/accuracy_ab3.jsonl 2> gpurun_out/r4/accuracy_ab3.log && timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_runtime.py tests/test_gpu_kernels.py tests/test_loopback_gpu.py -k "table2d or multistep or fp32 or chained or lds_poison" > gpurun_out/r4/gputests4.txt 2>&1; tail -4 gpurun_out/r4/gputests4.txt; cut -c1-250 gpurun_out/r4/accuracy_ab3.jsonl; python3 -c '
import json
for l in open("gpurun_out/table2d_phases_ab.jsonl"):
    r=json.loads(l); print(r.get("slice_arg"), r.get("phases_arg"), r.get("phases"), r.get("ms_per_integration"))
'
