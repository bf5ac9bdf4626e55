set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 240 python bench.py --steps 40 --warmup 8 --force-collective > gpurun_out/r4/fc.json 2> gpurun_out/r4/fc.log; echo rc=$?
python3 -c "
import json
js=json.loads(open('gpurun_out/r4/fc.json').read().strip().splitlines()[-1])
print('verified', js['verified'], js.get('transport_error'), js.get('rccl_transport'))
for k,v in js.items():
    if isinstance(v,dict) and 'verified' in v: print(k, v['verified'], json.dumps(v)[:400])
"
tail -5 gpurun_out/r4/fc.log
