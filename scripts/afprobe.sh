#!/bin/bash
# build libacmi.so variants with afactor_u8.hip compiled under extra defines into
# build_variants/<name>/ (CPU side; the objects of the other sources are reused)
#   bash scripts/afprobe.sh afp1:-DAF_PROBE=1 afd3:-DAF_DEPTH=3 "x:-DAF_PROBE=1 -DAF_DEPTH=3"
cd "$(dirname "$0")/../actor-critic_amd/csrc" || exit 1
make -s >/dev/null || exit 1
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  d=../../build_variants/$name; mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=on -fno-slp-vectorize \
    -Wno-unused-function $defs -c afactor_u8.hip -o $d/afactor_u8.o || exit 1
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libacmi.so build/net.o build/rl.o build/kfac.o \
    $d/afactor_u8.o build/atari.o || exit 1
done
