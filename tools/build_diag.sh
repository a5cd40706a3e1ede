#!/bin/bash
# Timing-study builds of libscde_hip.so with parts of k_boot2 compiled out
# (SCDE_BOOT_DIAG bits: 1 no multiplicity loads, 2 no column loads, 4 no exp, 8 no
# reductions).  Results are wrong by construction; load with SCDE_LIB=build_diag/libd<N>.so.
set -e
cd "$(dirname "$0")/../scde_amd/csrc"
make -s
mkdir -p ../../build_diag
for d in "$@"; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -DSCDE_BOOT_DIAG=$d \
    -c kernels.hip -o ../../build_diag/kernels_d$d.o &
done
wait
for d in "$@"; do
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../../build_diag/libd$d.so ../../build_diag/kernels_d$d.o engine.o bh.o prior.o wpca.o pagoda.o
done
