set -e
B=$GRAFT_REPO_ROOT/build/bin/miint
for n in 1e6 1e7 18e6 1e8 1e9; do $B bench --integrand table --n $n --iters 200 | tail -1; done
$B bench --integrand table --n 18e6 --iters 200 --grid 256 | tail -1
