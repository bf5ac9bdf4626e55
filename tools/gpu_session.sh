#!/usr/bin/env bash
# Run a sequence of GPU steps on the gpurun box, each under its own time limit, stopping at
# the first fault-like exit (timeout 124/137, abort 134, segfault 139, signal > 128).
# Ordinary test failures (exit 1/2/3) do not stop the session.
#
#   tools/gpu_session.sh "name:seconds:command" ...
# Output of each step: gpurun_out/<name>.txt ; summary: gpurun_out/session.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/session.txt
# Bring the in-tree build up to date from plain bash (no GPU initialised here), never from a
# profiled or GPU-initialised process: under rocprofv3 --pmc every child process initialises
# the GPU and exec'ing make/sh from it is refused on this pool.
# (build/obj is not shipped to the box, so `make -q` alone always reports stale objects: the
# in-tree extension and CLIs count as current when no source or build file is newer.)
# Every shipped artifact is checked on its own against the sources it is built from: `make
# ext` refreshes the .so but not the CLIs, so a source newer than ANY of them means a rebuild
# (miintrun is built from its one file and net.hpp only).
newer_src() {  # artifact, sources... -> true if a source is newer than the artifact
  local a="$1"; shift
  [ -n "$(find "$@" -newer "$a" -type f -print -quit)" ]
}
built_ok() {
  local so a; so=$(ls cuda_v_mpi_amd/_miint*.so 2>/dev/null | head -n 1)
  [ -n "$so" ] && [ -x build/bin/miintrun ] || return 1
  for a in "$so" build/bin/riemann build/bin/cintegrate build/bin/trainscan build/bin/miint; do
    [ -e "$a" ] || return 1
    newer_src "$a" csrc/include csrc/kernels csrc/runtime csrc/python csrc/cli Makefile && return 1
  done
  newer_src build/bin/miintrun csrc/cli/miintrun.cpp csrc/include/miint/net.hpp && return 1
  return 0
}
if ! built_ok && ! make -q all >/dev/null 2>&1; then
  echo "=== build out of date: make -j16 all" | tee -a gpurun_out/session.txt
  make -j16 all > gpurun_out/build.txt 2>&1 || { echo "=== build failed"; exit 1; }
fi
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"
  secs="${rest%%:*}"; cmd="${rest#*:}"
  start=$(date +%s)
  echo "=== $name ($secs s): $cmd" | tee -a gpurun_out/session.txt
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.txt" 2>&1
  rc=$?
  echo "=== $name rc=$rc elapsed=$(( $(date +%s) - start ))s" | tee -a gpurun_out/session.txt
  tail -n 5 "gpurun_out/$name.txt" | sed 's/^/    /' | tee -a gpurun_out/session.txt
  if [ "$rc" -ge 124 ]; then
    echo "=== stopping: fault-like exit $rc in $name" | tee -a gpurun_out/session.txt
    exit "$rc"
  fi
done
exit 0
