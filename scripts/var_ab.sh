#!/bin/bash
# bench.py at the default config and at configs[2] for library variants, alternating:
#   bash scripts/var_ab.sh <variant dir name> ...   (build_variants/<name>/libacmi.so; "intree")
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for v in "$@"; do
    lib=actor-critic_amd/libacmi.so; [ "$v" != intree ] && lib=build_variants/$v/libacmi.so
    for a in "" "--envs-per-gpu 32"; do
      ACMI_LIB=$lib timeout -k 10 120 python bench.py $a --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/vab.json 2> gpurun_out/vab.err || exit $?
      python - "$v" "$a" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/vab.json').read().strip().splitlines()[-1])
print('%-8s %-18s value %9.0f upd %.3f roll %.3f' % (sys.argv[1], sys.argv[2], d['value'], d['update_ms'], d['rollout_ms']))
PY
    done
  done
done
