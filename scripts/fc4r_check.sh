#!/bin/bash
# rollout fc4: staged gemm3 (ACMI_FC4R=0) vs fc4roll.hpp (1), bench per variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in 0 1 0 1; do
  ACMI_FC4R=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fc4r$v.json 2> gpurun_out/fc4r$v.err || exit $?
  python - "$v" <<'PY'
import json,sys
d=json.loads(open('gpurun_out/fc4r%s.json'%sys.argv[1]).read().strip().splitlines()[-1])
print('ACMI_FC4R', sys.argv[1], 'value %.0f upd %.3f roll %.3f' % (d['value'], d['update_ms'], d['rollout_ms']))
PY
done
