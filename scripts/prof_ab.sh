#!/bin/bash
# per-kernel A/B: rocprofv3 --kernel-trace --stats of a short bench with the base
# build (build_variants/base/libacmi.so) and with the tree's build; prints the
# kernels matching $1
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
for v in base tree; do
  lib=$root/actor-critic_amd/libacmi.so; [ $v = base ] && lib=$root/build_variants/base/libacmi.so
  ACMI_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/pab_$v" -o p --output-format csv \
    -- python3 "$root/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$root/gpurun_out/pab_$v.json" 2> "$root/gpurun_out/pab_$v.err" || exit $?
  f=$(find "$root/gpurun_out/pab_$v" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$1" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if sys.argv[2] in r['Name']:
        print(sys.argv[3], '%8.1f us x %s  %s' % (float(r['AverageNs']) / 1e3, r['Calls'], r['Name'][:90]))
PY
done
