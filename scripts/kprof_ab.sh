#!/bin/bash
# Per-kernel same-lease A/B: rocprofv3 --kernel-trace --stats of a short bench.py
# run with the in-tree libacmi.so and with ab/<name>/libacmi.so; prints one table
# (average us per launch, calls) of the kernels over 1 % of either run.
#   scripts/kprof_ab.sh "<bench args>" name
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
args=$1; name=$2
cd /tmp && export TMPDIR=/tmp
for v in tree "$name"; do
  lib=$root/actor-critic_amd/libacmi.so; [ "$v" != tree ] && lib=$root/ab/$v/libacmi.so
  ACMI_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$root/gpurun_out/kp_$v" -o p \
    --output-format csv -- python3 "$root/bench.py" $args --no-cpu-baseline --no-configs2 \
    > "$root/gpurun_out/kp_$v.json" 2> "$root/gpurun_out/kp_$v.err" || exit $?
done
python3 - "$root/gpurun_out" "$name" <<'PY'
import csv, glob, sys
d, name = sys.argv[1], sys.argv[2]
def load(v):
    f = glob.glob('%s/kp_%s/**/*kernel_stats.csv' % (d, v), recursive=True)[0]
    return {r['Name'][:100]: (float(r['AverageNs']) / 1e3, int(r['Calls']), float(r['Percentage']))
            for r in csv.DictReader(open(f))}
a, b = load('tree'), load(name)
print('%10s %10s %7s  %s' % ('tree us', name + ' us', 'calls', 'kernel'))
for k in sorted(set(a) | set(b), key=lambda k: -max(a.get(k, (0, 0, 0))[2], b.get(k, (0, 0, 0))[2])):
    if max(a.get(k, (0, 0, 0))[2], b.get(k, (0, 0, 0))[2]) < 1.0:
        continue
    print('%10.1f %10.1f %7d  %s' % (a.get(k, (0,))[0], b.get(k, (0,))[0], a.get(k, (0, 0))[1], k))
PY
