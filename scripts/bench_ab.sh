#!/bin/bash
# A/B of bench.py: base build (build_variants/base/libacmi.so, copied there from the
# base tree first) vs the tree's build, alternating; prints value / update / rollout
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for lib in build_variants/base/libacmi.so actor-critic_amd/libacmi.so; do
    ACMI_LIB=$lib timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
    python - "$lib" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'value %.0f upd %.3f roll %.3f' % (d['value'], d['update_ms'], d['rollout_ms']))
PY
  done
done
