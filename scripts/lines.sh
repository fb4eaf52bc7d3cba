#!/bin/bash
# bench.py lines, one per "<label>|<ACMI_LIB or empty>|<extra bench args>" spec, two rounds
#   scripts/lines.sh "<common bench args>" spec1 spec2 ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
common=$1; shift
for r in 1 2; do
  for spec in "$@"; do
    IFS='|' read -r label lib extra <<< "$spec"
    echo "== $label"
    ACMI_LIB="$lib" timeout -k 10 120 python bench.py $common $extra --no-cpu-baseline --no-configs2 \
      > gpurun_out/lines.json 2> gpurun_out/lines.err || { tail -5 gpurun_out/lines.err; exit 1; }
    python3 -c 'import json; d=json.loads(open("gpurun_out/lines.json").read().strip().splitlines()[-1]); print("value %.0f  ms %.3f  update %.3f (plain %.3f)  rollout %.3f  roofline-kernel %.4f ms" % (d["value"], d["ms_per_step"], d["update_ms"], d["update_ms_plain_iters"], d["rollout_ms"], d["roofline"]["avg_ms"] or 0))'
  done
done
