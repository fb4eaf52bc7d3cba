#!/bin/bash
# solo band backward timings (kbench, site 2 = the conv2 band kernel) under
# block-map / chunk / group-order variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "ACMI_BAND=0" "ACMI_BAND_MAP=1" "ACMI_BAND_MAP=0" "ACMI_BAND_CHUNKS=8" "ACMI_BAND_CHUNKS=16" \
         "ACMI_BAND_SORT=1" "ACMI_BAND_SORT=1 ACMI_BAND_CHUNKS=8" "ACMI_BAND_MAP=1 ACMI_BAND_SORT=1"; do
  echo "=== $v: $(env $v timeout -k 10 60 python scripts/kbench.py backward1 10240 2>&1 | tail -1)" || exit $?
done
