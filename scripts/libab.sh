#!/bin/bash
# A/B of the in-tree libacmi.so against build_variants/<name>/libacmi.so on one kbench command
#   scripts/libab.sh "<kbench args>" name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
args=$1; shift
for r in 1 2; do
  echo "== in-tree"; timeout -k 10 60 python scripts/kbench.py $args || exit $?
  for v in "$@"; do echo "== $v"; ACMI_LIB=build_variants/$v/libacmi.so timeout -k 10 60 python scripts/kbench.py $args || exit $?; done
done
