#!/bin/bash
# rocprofv3 kernel stats of one bench config under a library variant
#   bash scripts/prof_lib.sh <name> <lib path> <bench args...>   (outputs under gpurun_out/<name>/)
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=$1; lib=$2; shift 2
out="$root/gpurun_out/$name"; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
ACMI_LIB="$root/$lib" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof" -o prof --output-format csv -- \
  python3 "$root/bench.py" "$@" --steps 30 --warmup 5 --no-cpu-baseline > "$out/bench.json" 2> "$out/err.log" || exit $?
f=$(find "$out/prof" -name '*kernel_stats.csv' | head -1)
cp "$f" "$out/kernel_stats.csv"
python3 - "$out/kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('%8.1f us x %5s  %s' % (float(r['AverageNs']) / 1e3, r['Calls'], r['Name'][:90]))
PY
