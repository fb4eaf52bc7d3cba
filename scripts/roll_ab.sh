#!/bin/bash
# rollout / update ms of the default bench line under library variants (alternating)
#   scripts/roll_ab.sh intree name1 name2 ...   [BENCH_ARGS="--envs-per-gpu 32"]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != intree ] && lib="ACMI_LIB=build_variants/$v/libacmi.so"
    env $lib timeout -k 10 120 python bench.py $BENCH_ARGS --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/rab.json 2>/dev/null || exit 1
    python - "$v" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/rab.json').read().strip().splitlines()[-1])
print('%-8s value %8.0f upd %.3f roll %.3f band %.3f' % (sys.argv[1], d['value'], d['update_ms'], d['rollout_ms'], d['roofline']['avg_ms'] or 0))
PY
  done
done
