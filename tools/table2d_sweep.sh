for g in 4096 8192; do
  build/bin/miint table2d --grid $g --iters 200 || exit $?
  for w in 2 4 8; do build/bin/miint table2d --grid $g --slice 1/$w --iters 200 || exit $?; done
done
