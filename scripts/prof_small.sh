#!/bin/bash
# Kernel traces of the reference's own small configs: ACKTR 32 x 20 (BASELINE
# configs[2]) and A2C 32 x 5 (configs[1]): the bench line, a rocprofv3
# --kernel-trace --stats run of the same command, and the per-iteration
# launch / idle-gap table (scripts/trace_gaps.py).
#   bash scripts/prof_small.sh <name>      (outputs under gpurun_out/<name>/)
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=${1:-small}
cd "$root"
for cfg in "acktr32x20:--envs-per-gpu 32" "a2c32x5:--algo a2c --envs-per-gpu 32"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  out="$root/gpurun_out/$name/$tag"; mkdir -p "$out"
  echo "=== $tag bench"
  timeout -k 10 200 python3 bench.py $args --steps 50 --warmup 10 --no-cpu-baseline --no-configs2 > "$out/bench.json" 2> "$out/bench.err" || exit $?
  tail -1 "$out/bench.json" | cut -c1-300
  echo "=== $tag rocprofv3"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof" -o prof \
    --output-format csv -- python3 "$root/bench.py" $args --steps 30 --warmup 5 --no-cpu-baseline --no-configs2 \
    > "$out/prof_bench.json" 2> "$out/prof.err") || exit $?
  cp "$(find "$out/prof" -name '*kernel_stats.csv' | head -1)" "$out/kernel_stats.csv"
  cp "$(find "$out/prof" -name '*kernel_trace.csv' | head -1)" "$out/kernel_trace.csv"
  python3 scripts/trace_gaps.py "$out/kernel_trace.csv" > "$out/gaps.md" || exit $?
  head -12 "$out/gaps.md"
done
exit 0
