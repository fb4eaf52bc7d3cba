#!/bin/bash
# A/B of the K-FAC inverse: base build (build_variants/base/libacmi.so, copied there
# from the base tree first) vs the tree's
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  ACMI_LIB=build_variants/base/libacmi.so timeout -k 10 60 python scripts/inv_bench.py || exit $?
  timeout -k 10 60 python scripts/inv_bench.py || exit $?
done
