#!/bin/bash
# A/B an env toggle at configs[2] and the default config, alternating
cd "${GRAFT_REPO_ROOT}"
var=$1; shift
for i in 1 2 3; do
  for v in "$@"; do
    for a in "--envs-per-gpu 32" "--algo a2c --envs-per-gpu 32" ""; do
      env $var=$v timeout -k 10 120 python bench.py $a --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/vab.json 2> gpurun_out/vab.err || exit $?
      python - "$v" "$a" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/vab.json').read().strip().splitlines()[-1])
print('%-6s %-30s value %9.0f upd %.3f roll %.3f' % (sys.argv[1], sys.argv[2], d['value'], d.get('update_ms',0), d.get('rollout_ms',0)))
PY
    done
  done
done
