#!/bin/bash
# acmi_kfac_inverse time (scripts/inv_bench.py) with the in-tree build and ab/<name> builds, two rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  echo "== in-tree"; timeout -k 10 60 python scripts/inv_bench.py || exit $?
  for v in "$@"; do echo "== $v"; ACMI_LIB=ab/$v/libacmi.so timeout -k 10 60 python scripts/inv_bench.py || exit $?; done
done
