#!/bin/bash
# The round's whole measurement package in one GPU call: the default bench line
# with its rocprofv3 stats and FETCH/WRITE passes, the small-config traces, and the
# bench line at every BASELINE config (each step under its own time limit; the
# first failing step ends the call).   bash scripts/round_package.sh <name>
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=${1:-pkg}
cd "$root"
bash scripts/profile_package.sh "$name" || exit $?
bash scripts/prof_small.sh "$name/small" || exit $?
bash scripts/config_lines.sh "${name}_lines" || exit $?
exit 0
