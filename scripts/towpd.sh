#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for pd in 2 3 4; do echo "PD=$pd"; ACMI_TOWER_PD=$pd timeout -k 10 60 python scripts/kbench.py forward 512 || exit $?; done
