#!/bin/bash
# bench with / without the fused conv tower (rollout ms is where it shows)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "ACMI_TOWER=1" "ACMI_TOWER=0"; do
  env $v timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/tw_$v.json 2> gpurun_out/tw_$v.err || exit $?
  python - "$v" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/tw_%s.json'%sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], 'value %.0f upd %.3f roll %.3f' % (d['value'], d['update_ms'], d['rollout_ms']))
PY
done
