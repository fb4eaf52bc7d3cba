#!/bin/bash
# conv tower launch (kbench forward, site 3) vs batch, 4-wave and 16-wave bodies
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for B in 32 128 512; do
    ACMI_WIDE_TOWER_MAX=0 timeout -k 10 60 python scripts/kbench.py forward $B 2>/dev/null | sed "s/^/4wave /" || exit 1
  done
  timeout -k 10 60 python scripts/kbench.py forward 32 2>/dev/null | sed "s/^/wide /" || exit 1
done
