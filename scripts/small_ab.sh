#!/bin/bash
# BASELINE configs[2] (ACKTR 32 x 20) and configs[1] (A2C 32 x 5) bench lines
# under environment variants:  scripts/small_ab.sh "VAR=x VAR2=y" "VAR=z" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
for v in "$@"; do
  for a in "--envs-per-gpu 32" "--algo a2c --envs-per-gpu 32"; do
    env $v timeout -k 10 100 python bench.py $a --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/sab.json 2>/dev/null || exit 1
    python - "$v" "$a" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/sab.json').read().strip().splitlines()[-1])
print('%-50s %-32s value %8.0f upd %.3f roll %.3f' % (sys.argv[1], sys.argv[2], d['value'], d['update_ms'], d['rollout_ms']))
PY
  done
done
done
