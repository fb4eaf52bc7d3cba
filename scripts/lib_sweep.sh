#!/bin/bash
# A command under several builds of libacmi.so (build_variants/<name>/libacmi.so),
# alternating twice:  bash scripts/lib_sweep.sh "<command>" name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cmd=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    echo "--- $v (rep $rep)"
    ACMI_LIB=build_variants/$v/libacmi.so timeout -k 10 120 bash -c "$cmd" 2>&1 | grep -v amdgpu.ids | tail -2 || exit $?
  done
done
