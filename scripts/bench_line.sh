#!/bin/bash
# one bench.py run (extra args passed through), summarised: value, roofline kernel ms, update ms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 150 python bench.py --no-cpu-baseline "$@" > gpurun_out/bl.json 2> gpurun_out/bl.err || exit $?
python3 - <<'PY'
import json
d = json.loads(open('gpurun_out/bl.json').read().strip().splitlines()[-1])
print('value %.0f  roofline-kernel %.4f ms  update plain %.3f inv %.3f  rollout %.3f' % (
    d['value'], d['roofline']['avg_ms'], d['update_ms_plain_iters'], d['update_ms_inverse_iters'], d['rollout_ms']))
PY
