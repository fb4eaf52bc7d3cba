#!/bin/bash
# libacmi.so variants with net.hip compiled under extra defines into ab/<name>/
# (git-ignored scratch; the other objects reused) for same-lease A/Bs
#   bash scripts/net_variant.sh d6:-DACMI_SPLIT_DEPTH=6 ...
cd "$(dirname "$0")/../actor-critic_amd/csrc" || exit 1
make -s >/dev/null || exit 1
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  d=../../ab/$name; mkdir -p $d
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=on -fno-slp-vectorize \
    -Wno-unused-function -Wno-pass-failed $defs -c net.hip -o $d/net.o || exit 1
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $d/libacmi.so $d/net.o build/rl.o build/kfac.o \
    build/afactor_u8.o build/atari.o || exit 1
  rm -f $d/net.o
done
