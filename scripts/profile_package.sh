#!/bin/bash
# Round measurement package: default bench line, rocprofv3 --kernel-trace --stats
# of the same command (short), and FETCH/WRITE PMC passes for the roofline kernel.
#   bash scripts/profile_package.sh <name>      (outputs under gpurun_out/<name>/)
set -o pipefail
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
name=${1:-pkg}
out="$root/gpurun_out/$name"; mkdir -p "$out"
cd "$root"
echo "=== bench"
timeout -k 10 300 python3 bench.py > "$out/bench_default.json" 2> "$out/bench.err" || exit $?
tail -1 "$out/bench_default.json" | cut -c1-400
cd /tmp && export TMPDIR=/tmp
echo "=== rocprofv3 stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o prof --output-format csv \
  -- python3 "$root/bench.py" --steps 10 --warmup 2 --no-cpu-baseline --no-configs2 > "$out/prof_bench.json" 2> "$out/prof.err" || exit $?
f=$(find "$out/prof" -name '*kernel_stats.csv' | head -1)
cp "$f" "$out/kernel_stats.csv"
python3 "$root/scripts/prof_summary.py" "$out/kernel_stats.csv" "rocprofv3 --kernel-trace --stats, bench.py --steps 10 --warmup 2 --no-cpu-baseline (12 iterations), ACKTR 512x20, 1x MI355X" 12 > "$out/summary.md"
trace=$(find "$out/prof" -name '*kernel_trace.csv' | head -1)
cp "$trace" "$out/kernel_trace.csv"
echo "=== pmc"
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pmc -d "$out/pmc/$pmc" -o "$pmc" --output-format csv \
    -- python3 "$root/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-configs2 > "$out/pmc_$pmc.log" 2>&1 || exit $?
done
exit 0
