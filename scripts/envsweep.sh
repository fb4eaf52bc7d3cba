#!/bin/bash
# bench under several environment settings: scripts/envsweep.sh "A=1 B=2" "A=0" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/sw$i.json 2> gpurun_out/sw$i.err || exit $?
  python - "$cfg" gpurun_out/sw$i.json <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print('%-50s value %9.0f  upd %.3f plain %.3f inv %.3f roll %.3f' % (sys.argv[1], d['value'], d['update_ms'], d['update_ms_plain_iters'], d['update_ms_inverse_iters'], d['rollout_ms']))
PY
done
