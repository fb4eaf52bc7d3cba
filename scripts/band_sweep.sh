#!/bin/bash
# solo band backward timings (kbench band: conv2 band kernel vs its MFMA bound)
# under plan variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "ACMI_BAND_CAP=16" "ACMI_BAND_CAP=8" "ACMI_BAND_CAP=12" "ACMI_BAND_CAP=8 ACMI_BAND_MAP=1" "ACMI_BAND_CAP=8 ACMI_BAND_SORT=0" "ACMI_BAND_CAP=4"; do
  echo "=== $v"
  env $v timeout -k 10 100 python scripts/kbench.py band 2>&1 | grep -v amdgpu.ids | tail -2 || exit $?
done
