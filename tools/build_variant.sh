#!/bin/bash
# Study builds of libscde_hip.so with kernels.hip compiled under extra -D flags:
#   tools/build_variant.sh NAME "-DSCDE_KT_STAMP=1" [NAME2 "FLAGS2" ...]
# writes diag/libNAME.so (diag/ travels with gpurun; load with SCDE_LIB=diag/libNAME.so).
set -e
cd "$(dirname "$0")/../scde_amd/csrc"
make -s
mkdir -p ../../diag
args=("$@")
for ((i = 0; i < ${#args[@]}; i += 2)); do
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include ${args[i+1]} \
    -c kernels.hip -o ../../diag/kernels_${args[i]}.o &
done
wait
for ((i = 0; i < ${#args[@]}; i += 2)); do
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../../diag/lib${args[i]}.so ../../diag/kernels_${args[i]}.o engine.o bh.o prior.o wpca.o pagoda.o
done
