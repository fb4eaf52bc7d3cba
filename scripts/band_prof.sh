#!/bin/bash
# solo kernel times of the backward (kbench backward1) in band / patch modes and
# band chunk variants, plus FETCH/WRITE PMC passes of the band backward
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/bandprof"; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
run() {  # name env...
  local name=$1; shift
  echo "=== $name"
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out/$name" -o "$name" --output-format csv \
    -- python3 "$root/scripts/kbench.py" backward1 10240 > "$out/$name.log" 2>&1 || return $?
  f=$(find "$out/$name" -name '*kernel_stats.csv' | head -1)
  python3 "$root/scripts/prof_summary.py" "$f" "$name" 5 > "$out/$name.md"
}
run band ACMI_BAND=1 || exit $?
run patch ACMI_BAND=0 || exit $?
run band_c2 ACMI_BAND_CHUNKS=2 || exit $?
run band_c8 ACMI_BAND_CHUNKS=8 || exit $?
for pmc in FETCH_SIZE WRITE_SIZE; do
  echo "=== pmc $pmc"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc -d "$out/pmc_$pmc" -o "pmc_$pmc" --output-format csv \
    -- python3 "$root/scripts/kbench.py" backward1 10240 > "$out/pmc_$pmc.log" 2>&1 || exit $?
done
exit 0
