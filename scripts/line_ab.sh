#!/bin/bash
# Same-lease A/B of bench.py lines: in-tree libacmi.so vs ab/<name>/libacmi.so,
# each under the listed ACMI_CONCURRENT_STATS settings, two rounds.
#   scripts/line_ab.sh "<bench args>" "<conc settings, e.g. '0 1' or 'auto'>" name1 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
args=$1; concs=$2; shift 2
one() {  # lib conc
  local lib=$1 c=$2
  local env=()
  [ "$c" != auto ] && env+=(ACMI_CONCURRENT_STATS=$c)
  echo "== lib=${lib:-in-tree} conc=$c"
  env ACMI_LIB="$lib" "${env[@]}" timeout -k 10 120 python bench.py $args --no-cpu-baseline --no-configs2 \
    > gpurun_out/line_ab.json || return 1
  python3 -c 'import json; d=json.loads(open("gpurun_out/line_ab.json").read().strip().splitlines()[-1]); print("value %.0f  ms %.3f  update %.3f (plain %.3f)  rollout %.3f  roofline-kernel %.4f ms" % (d["value"], d["ms_per_step"], d["update_ms"], d["update_ms_plain_iters"], d["rollout_ms"], d["roofline"]["avg_ms"] or 0))'
}
for r in 1 2; do
  for c in $concs; do
    one "" $c || exit 1
    for v in "$@"; do one "ab/$v/libacmi.so" $c || exit 1; done
  done
done
