set -e
for a in fused lookback onepass; do build/bin/trainscan --algo $a --iters 50 --json | tail -1; done
build/bin/miint table2d --grid 4096 --iters 200
build/bin/miint table2d --grid 8192 --iters 200
