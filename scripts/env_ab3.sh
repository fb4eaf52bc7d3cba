#!/bin/bash
# same-lease A/B of one environment switch on the default bench line (two rounds)
#   bash scripts/env_ab3.sh VAR "v0 v1" [bench args]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
var=$1; vals=$2; shift 2
for r in 1 2; do
  for v in $vals; do
    env $var=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-configs2 "$@" > gpurun_out/envab.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/envab.json').read().strip().splitlines()[-1]); print('$var=$v', round(d['value']), 'upd %.3f roll %.3f band %.3f' % (d['update_ms'], d['rollout_ms'], d['roofline']['avg_ms']))"
  done
done
