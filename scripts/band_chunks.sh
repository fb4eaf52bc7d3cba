#!/bin/bash
# conv2 band launch (kbench backward1x, site 2) under forced chunk counts
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for c in "$@"; do
    ACMI_BAND_CHUNKS=$c timeout -k 10 60 python scripts/kbench.py backward1x 2>/dev/null | sed "s/^/chunks=$c /" || exit 1
  done
done
