#!/bin/bash
# kernel-trace averages of one kernel across libacmi.so variants on one kbench command
#   scripts/libprof.sh "<kbench args>" <kernel-name regex> name1 name2 ...  (in-tree lib first)
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
args=$1; pat=$2; shift 2
cd /tmp && export TMPDIR=/tmp
for v in tree "$@"; do
  out="$root/gpurun_out/libprof/$v"; rm -rf "$out"; mkdir -p "$out"
  lib=""; [ "$v" != tree ] && lib="$root/build_variants/$v/libacmi.so"
  ACMI_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out" -o p --output-format csv \
    -- python3 "$root/scripts/kbench.py" $args > "$out/log" 2>&1 || exit $?
  f=$(find "$out" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$pat" "$v" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[2], r['Name']):
        print('%-8s %8.1f us  x%s  %s' % (sys.argv[3], float(r['AverageNs']) / 1e3, r['Calls'], r['Name'][:70]))
PY
done
