#!/bin/bash
# 4-wave tower launch (kbench forward, site 3) at B = 32 and 512 under probe builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != intree ] && lib="ACMI_LIB=build_variants/$v/libacmi.so"
    for B in 32 512; do
      env $lib timeout -k 10 60 python scripts/kbench.py forward $B 2>/dev/null | sed "s/^/$v /" || exit 1
    done
  done
done
