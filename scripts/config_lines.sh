#!/bin/bash
# The bench line at every BASELINE.json config that fits one GPU, each with its
# cpu_baseline at the same config:  bash scripts/config_lines.sh <outdir-name>
root="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
out="$root/gpurun_out/${1:-lines}"; mkdir -p "$out"
cd "$root"
run() {
  local name=$1; shift
  echo "=== $name: bench.py $*"
  timeout -k 10 240 python3 bench.py "$@" > "$out/$name.json" 2> "$out/$name.err" || return $?
  tail -1 "$out/$name.json" | cut -c1-260
}
run configs3_shard_acktr_512x20 || exit $?
run configs2_acktr_32x20 --envs-per-gpu 32 --steps 50 --warmup 10 || exit $?
run configs1_a2c_32x5 --algo a2c --envs-per-gpu 32 --steps 100 --warmup 10 || exit $?
run configs4_shard_bf16_1024x20_a18 --forward bf16 --num-actions 18 --envs-per-gpu 1024 || exit $?
run configs4_mixed_atari57_1024x20_a18_bf16 --forward bf16 --num-actions 18 --envs-per-gpu 1024 --games atari57 \
  --cpu-iters 2 || exit $?
exit 0
