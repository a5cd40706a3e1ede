#!/bin/bash
# Study builds of libscde_hip.so with kernels.hip compiled under extra -D flags (or from a git
# revision): tools/variant.sh NAME "FLAGS" [NAME2 "FLAGS2" ...]; FLAGS "@REV" builds kernels.hip as
# of git revision REV.  Writes var/libNAME.so (var/ travels with gpurun; SCDE_LIB=var/libNAME.so).
set -e
cd "$(dirname "$0")/../scde_amd/csrc"
make -s
mkdir -p ../../var
args=("$@")
for ((i = 0; i < ${#args[@]}; i += 2)); do
  f=${args[i+1]}; src=kernels.hip
  if [[ $f == @* ]]; then src=../../var/kernels_${args[i]}.hip; git show ${f#@}:scde_amd/csrc/kernels.hip > $src; f=""; fi
  hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -I../../include -I. $f -c $src -o ../../var/kernels_${args[i]}.o &
done
wait
for ((i = 0; i < ${#args[@]}; i += 2)); do
  hipcc -shared -fPIC --offload-arch=gfx950 -o ../../var/lib${args[i]}.so ../../var/kernels_${args[i]}.o engine.o bh.o prior.o wpca.o pagoda.o
done
