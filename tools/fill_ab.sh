#!/usr/bin/env bash
# A/B of interp_fill builds kept under variants/ (each a full _miint .so): alternates them
# through tools/interp_fill_probe.py and restores the in-tree build afterwards.
set -e
SO=$(ls cuda_v_mpi_amd/_miint*.so)
cp "$SO" /tmp/orig.so
for pass in 1 2 3; do
  for f in variants/*.so; do
    cp "$f" "$SO"
    printf '%s pass%s ' "$(basename "$f" .so)" "$pass"
    timeout -k 10 60 python -u tools/interp_fill_probe.py 300 | grep '^{'
  done
done
cp /tmp/orig.so "$SO"
