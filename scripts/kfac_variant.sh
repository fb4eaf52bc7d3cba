#!/bin/bash
# build libacmi.so variants with kfac.hip compiled under extra defines into
# build_variants/<name>/ (the other objects reused)
#   bash scripts/kfac_variant.sh gp0:-DACMI_GJ_PAIRS=0
cd "$(dirname "$0")/../actor-critic_amd/csrc" || exit 1
make -s >/dev/null || exit 1
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  d=../../build_variants/$name; mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=on -fno-slp-vectorize \
    -Wno-unused-function -Wno-pass-failed $defs -c kfac.hip -o $d/kfac.o || exit 1
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libacmi.so build/net.o build/rl.o $d/kfac.o \
    build/afactor_u8.o build/atari.o || exit 1
done
