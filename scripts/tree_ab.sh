#!/bin/bash
# A/B of the default bench line: the tree under build_variants/basetree (its own
# package + libacmi.so) against this tree, alternating, on one lease
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2 3; do
  for b in build_variants/basetree/bench.py bench.py; do
    timeout -k 10 120 python $b --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab.json 2> gpurun_out/ab.err || exit $?
    python - "$b" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'value %.0f upd %.3f roll %.3f band %.3f' % (d['value'], d['update_ms'], d['rollout_ms'], d['roofline']['avg_ms']))
PY
  done
done
