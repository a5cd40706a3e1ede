#!/bin/bash
# config 4 bootstrap: kernel time and counter bytes (FETCH_SIZE) per gene order / jp chunking:
#   bash tools/c4_order.sh OUTDIR "to3:tile_order=3 to1:tile_order=1 ..."
set -o pipefail
out=${1:-gpurun_out/c4}; specs=${2:-"to3:tile_order=3 to1:tile_order=1"}
mkdir -p $out
for spec in $specs; do
  name=${spec%%:*}; opts=${spec#*:}
  optargs=""; for o in ${opts//,/ }; do optargs="$optargs --opt $o"; done
  KT_LIBS="$name:" KT_ARGS="--config 4 --opt modes_overlap=0 $optargs" bash tools/ktrace_ab.sh $out/kt "k_boot_gene|k_boot_tiles|k_boot2|k_sum" || exit 1
  PMC_LIBS="$name:" PMC="FETCH_SIZE" PMC_ARGS="--config 4 --opt modes_overlap=0 $optargs" bash tools/pmc_ab.sh $out/pmc "k_boot_gene" || exit 1
done
