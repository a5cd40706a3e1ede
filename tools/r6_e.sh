#!/bin/bash
set -o pipefail
D=gpurun_out/r6e; mkdir -p $D
KT_LIBS="old:var/libold.so cur: w2:var/libw2.so w2nosb:var/libw2nosb.so nosb:var/libnosb.so" bash tools/ktrace_ab.sh $D/kt k_tables_reg || exit 1
AB_LIBS="gate:: nogate::boot_gate=0" AB_ARGS="--config 3 --shard-of 8" AB_REPS=3 bash tools/ab.sh $D/s8 || exit 1
