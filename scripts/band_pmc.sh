#!/bin/bash
# PMC passes over the band-mode backward (kbench backward1), one rocprofv3 run per pass
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$root"
PASSES="${PASSES:-sq lds tcc fetch write}" bash scripts/pmc.sh pmc_band scripts/kbench.py backward1 10240 || exit $?
python3 scripts/pmc_table.py gpurun_out/pmc_band > gpurun_out/pmc_band/table.txt 2>&1
exit 0
