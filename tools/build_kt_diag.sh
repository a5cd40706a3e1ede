#!/bin/bash
# Timing-study builds of libscde_hip.so with parts of k_tables compiled out
# (SCDE_KT_DIAG bits: 1 trivial dnbinom, 2 no exp, 4 no log, 8 no stores).  Results are
# wrong by construction; load with SCDE_LIB=build_diag/libkt<N>.so.
set -e
cd "$(dirname "$0")/../scde_amd/csrc"
make -s
mkdir -p ../../build_diag
for d in "$@"; do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -DSCDE_KT_DIAG=$d \
    -c kernels.hip -o ../../build_diag/kernels_kt$d.o &
done
wait
for d in "$@"; do
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../../build_diag/libkt$d.so ../../build_diag/kernels_kt$d.o engine.o bh.o prior.o wpca.o pagoda.o
done
