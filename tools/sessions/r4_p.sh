# round 4 session P: multi-step replays past residency (8192^2, 6144^2) vs chained replays
set -uo pipefail
mkdir -p gpurun_out/r4
out=gpurun_out/r4/t2d_ms_any_ab.jsonl; : > $out
for rep in 1 2; do for g in 8192 6144; do
  for dir in build/bin build/ab_msany/bin; do
    for extra in "" "--no-multistep"; do
      [ "$dir" = build/ab_msany/bin ] && [ -n "$extra" ] && continue
      line=$(timeout -k 10 60 $dir/miint table2d --grid $g --iters 640 $extra | grep '^{' | tail -1) || exit 1
      echo "{\"rep\": $rep, \"build\": \"$dir\", \"extra\": \"$extra\", ${line#\{}" >> $out
    done
  done
done; done
python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$out'):
    r=json.loads(l); d[(r['grid'], r['build'], r['extra'], r['multistep'], r['phases'], r['step_streams'])].append((round(r['ms_per_integration']*1e3,3), r.get('rel_err_vs_oracle')))
for k in sorted(d): print(k, d[k])"
