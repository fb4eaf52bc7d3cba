#!/bin/bash
# Same-lease A/B of the in-tree libacmi.so against ab/<name>/libacmi.so (ab/ is
# git-ignored scratch) on one kbench command, alternating, two rounds
#   scripts/ab.sh "<kbench args>" name1 name2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
args=$1; shift
for r in 1 2; do
  echo "== in-tree"; timeout -k 10 90 python scripts/kbench.py $args || exit $?
  for v in "$@"; do echo "== $v"; ACMI_LIB=ab/$v/libacmi.so timeout -k 10 90 python scripts/kbench.py $args || exit $?; done
done
