#!/bin/bash
# tower kernel: timing + PMC passes (kbench forward at the rollout batch)
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
timeout -k 10 60 python scripts/kbench.py forward 512 || exit $?
PASSES="${PASSES:-sq lds}" bash scripts/pmc.sh pmc_tower scripts/kbench.py forward 512 || exit $?
python3 scripts/pmc_table.py gpurun_out/pmc_tower > gpurun_out/pmc_tower/table.txt 2>&1
exit 0
