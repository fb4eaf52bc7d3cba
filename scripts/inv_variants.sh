#!/bin/bash
# K-FAC inverse timing + output hash (scripts/inv_bench.py) for the in-tree
# library and build_variants/<name>/libacmi.so
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for v in intree "$@"; do
    lib=""; [ "$v" != intree ] && lib="ACMI_LIB=build_variants/$v/libacmi.so"
    env $lib timeout -k 10 60 python scripts/inv_bench.py 2>/dev/null | sed "s/^/$v /" || exit 1
  done
done
