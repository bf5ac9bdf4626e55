# round 4 session F: 16 auto phases at HEAD (2-D tests incl. 16 / 32 phases bitwise), 16 vs 32
# phases on the whole field and slices, then the PMC roofline of the hot kernels at HEAD
set -uo pipefail
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread \
  tests/test_gpu_runtime.py tests/test_gpu_kernels.py tests/test_lds_poison_gpu.py -k "table2d or poison" \
  > gpurun_out/r4/gputests_f.txt 2>&1
rc=$?
[ $rc -le 1 ] || { tail -40 gpurun_out/r4/gputests_f.txt; exit $rc; }
grep -E "FAILED|^E " gpurun_out/r4/gputests_f.txt | cut -c1-300 || true
tail -2 gpurun_out/r4/gputests_f.txt
[ $rc -eq 0 ] || exit 1
out=gpurun_out/r4/t2d_phases_16_32.jsonl; : > $out
for rep in 1 2; do for sl in full 0/2 0/4 0/8; do for ph in 16 32; do
  extra=(); [ "$sl" != full ] && extra=(--slice "$sl")
  line=$(timeout -k 10 60 build/bin/miint table2d --grid 4096 --iters 640 --phases $ph "${extra[@]}" | grep '^{' | tail -1) || exit 1
  echo "{\"rep\": $rep, \"slice_arg\": \"$sl\", \"phases_arg\": $ph, ${line#\{}" >> $out
done; done; done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$out'):
    r=json.loads(l); d[(r['slice_arg'],r['phases'])].append(round(r['ms_per_integration']*1e3,3))
for k in sorted(d): print(k,d[k])"
bash tools/sessions/r4_pmc.sh > gpurun_out/r4/pmc_session.txt 2>&1 || { tail -20 gpurun_out/r4/pmc_session.txt; exit 1; }
tail -30 gpurun_out/r4/roofline.md
