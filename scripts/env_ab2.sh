#!/bin/bash
# A/B an env knob at configs[2] and the default config, alternating:
#   bash scripts/env_ab2.sh <VAR> <value> ...   ("-" = unset)
cd "${GRAFT_REPO_ROOT}"
var=$1; shift
for i in 1 2; do
  for v in "$@"; do
    for a in "--envs-per-gpu 32" ""; do
      if [ "$v" = - ]; then e=""; else e="$var=$v"; fi
      env $e timeout -k 10 120 python bench.py $a --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/vab.json 2> gpurun_out/vab.err || exit $?
      python - "$v" "$a" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/vab.json').read().strip().splitlines()[-1])
print('%-6s %-20s value %9.0f upd %.3f roll %.3f' % (sys.argv[1], sys.argv[2], d['value'], d.get('update_ms',0), d.get('rollout_ms',0)))
PY
    done
  done
done
