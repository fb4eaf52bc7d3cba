#!/bin/bash
# A/B: conv tower kernel time at the rollout batch, base build vs the tree's build
# (first: mkdir -p build_variants/base && cp actor-critic_amd/libacmi.so build_variants/base/ from the base tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  ACMI_LIB=build_variants/base/libacmi.so timeout -k 10 60 python scripts/kbench.py forward 512 || exit $?
  timeout -k 10 60 python scripts/kbench.py forward 512 || exit $?
done
