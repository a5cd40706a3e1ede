#!/bin/bash
# Timing-study builds of libscde_hip.so with parts of k_boot_tiles8 compiled out
# (SCDE_TILE_DIAG bits: 1 bounds only, 2 rows without bounds).  Results are wrong by
# construction; load with SCDE_LIB=diag/libt<N>.so (diag/ travels with gpurun, build_diag/ does not).
set -e
cd "$(dirname "$0")/../scde_amd/csrc"
make -s
mkdir -p ../../diag
for d in "$@"; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -DSCDE_TILE_DIAG=$d \
    -c kernels.hip -o ../../diag/kernels_t$d.o &
done
wait
for d in "$@"; do
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../../diag/libt$d.so ../../diag/kernels_t$d.o engine.o bh.o prior.o wpca.o pagoda.o
done
