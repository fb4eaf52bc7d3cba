#!/bin/bash
# rocprofv3 kernel trace of a short bench run under extra environment settings:
#   bash scripts/prof_env.sh <name> [VAR=value ...]   (outputs under gpurun_out/<name>/)
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=$1; shift
for kv in "$@"; do export "$kv"; done
out="$root/gpurun_out/$name"; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$out/prof" -o prof --output-format csv \
  -- python3 "$root/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$out/bench.json" 2> "$out/prof.err" || exit $?
cp "$(find "$out/prof" -name '*kernel_stats.csv' | head -1)" "$out/kernel_stats.csv"
cp "$(find "$out/prof" -name '*kernel_trace.csv' | head -1)" "$out/kernel_trace.csv"
rm -rf "$out/prof"
tail -c 600 "$out/bench.json"
