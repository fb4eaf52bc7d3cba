#!/bin/bash
# tower timing probes: libacmi built with -DTPROBE=<bits> into build_variants/tp<bits>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  echo "TPROBE=$v"; ACMI_LIB=build_variants/tp$v/libacmi.so timeout -k 10 60 python scripts/kbench.py forward 512 || exit $?
done
