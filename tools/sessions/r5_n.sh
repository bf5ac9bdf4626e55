#!/bin/bash
# r5 session N: 2-D replay size sweep (integrations per multi-step replay) and step phases at
# the auto replay size, whole 4096^2 field and its 1/2, 1/4, 1/8 row slices
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5
mkdir -p $O
: > $O/n_t2d_steps.jsonl
run() {  # tag, args
  local line
  line=$(timeout -k 10 90 build/bin/miint table2d --grid 4096 $2 | grep '^{' | tail -1) || return 1
  echo "{\"tag\": \"$1\", ${line#\{}" >> $O/n_t2d_steps.jsonl
}
for rep in 1 2; do
  for gs in 32 64 128 256 512 1024; do
    run "full_gs$gs" "--graph-steps $gs" || exit 1
    run "s8_gs$gs" "--slice 0/8 --graph-steps $gs" || exit 1
  done
  for sl in 0/2 0/4; do
    for gs in 128 256 512 1024; do run "s${sl#0/}_gs$gs" "--slice $sl --graph-steps $gs" || exit 1; done
  done
  for ph in 8 16 32; do
    run "full_auto_ph$ph" "--phases $ph" || exit 1
    run "s8_auto_ph$ph" "--slice 0/8 --phases $ph" || exit 1
  done
done
echo "exit 0"
