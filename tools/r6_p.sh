#!/bin/bash
set -o pipefail
D=gpurun_out/r6p; mkdir -p $D
rc=0

[ $rc -ne 0 ] && { grep -E "FAILED|Error" $D/gputests.log | head -20; exit 1; }
AB_LIBS="old:var/libold.so new:" AB_REPS=2 bash tools/ab.sh $D/ab3 || exit 1
AB_LIBS="old:var/libold.so new:" AB_ARGS="--config 3 --shard-of 8" AB_REPS=2 bash tools/ab.sh $D/s8 || exit 1
