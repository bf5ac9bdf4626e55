# round 4 session L: settled one-shot grid / block sweep (graph_poll and direct_poll)
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python tools/one_shot_grid.py 60 graph_poll > gpurun_out/r4/one_shot_grid_settled.jsonl 2> gpurun_out/r4/one_shot_grid.log || { tail -5 gpurun_out/r4/one_shot_grid.log; exit 1; }
timeout -k 10 300 python tools/one_shot_grid.py 60 direct_poll >> gpurun_out/r4/one_shot_grid_settled.jsonl 2>> gpurun_out/r4/one_shot_grid.log || { tail -5 gpurun_out/r4/one_shot_grid.log; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r4/one_shot_grid_settled.jsonl'):
    r=json.loads(l); print(r['mode'], r['block'], r['grid'], round(r['median_us'],2), round(r['device_median_us'],2))"
