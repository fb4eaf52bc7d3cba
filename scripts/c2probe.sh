#!/bin/bash
# convt2 timing probes (kbench backward, site = conv2 dX); dbg bits: 1 no dY loads,
# 2 no weight staging, 4 no MFMA, 8 no epilogue, 16 no stores, 32 no mask loads,
# 64 no LDS reads, 128 no LDS writes, 256 no barriers
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for d in 0 1 2 4 8 15; do
  echo "dbg=$d"; ACMI_C2DBG=$d timeout -k 10 60 python scripts/kbench.py c2 10240 || exit $?
done
