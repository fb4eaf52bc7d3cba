#!/bin/bash
# Band-kernel measurement: HIP-event timing of the conv2 band launch (kbench
# backward1x) and the PMC passes of scripts/band_pmc.sh, into gpurun_out/<name>/
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=${1:-band}
out="$root/gpurun_out/$name"; mkdir -p "$out"
cd "$root"
timeout -k 10 120 python3 scripts/kbench.py backward1x 10240 > "$out/time.log" 2>&1 || exit $?
cat "$out/time.log"
PASSES="${PASSES:-sq lds tcc fetch write}" bash scripts/pmc.sh "$name/pmc" scripts/kbench.py backward1 10240 || exit $?
python3 scripts/pmc_table.py "$out/pmc" > "$out/table.txt" 2>&1
grep -A12 band_kernel "$out/table.txt" || true
exit 0
