#!/bin/bash
# conv2 band launch (kbench band at M = 10240, site 2) under probe builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != intree ] && lib="ACMI_LIB=build_variants/$v/libacmi.so"
    env $lib timeout -k 10 60 python scripts/kbench.py backward1x 10240 2>/dev/null | sed "s/^/$v /" || exit 1
  done
done
