#!/bin/bash
# rocprofv3 kernel stats of scripts/inv_bench.py (the K-FAC inverse launches)
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/inv_prof"; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out" -o prof --output-format csv -- \
  python3 "$root/scripts/inv_bench.py" > "$out/run.log" 2>&1 || exit $?
f=$(find "$out" -name '*kernel_stats.csv' | head -1)
cut -d, -f1-8 "$f" | head -12
