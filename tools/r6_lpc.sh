#!/bin/bash
set -o pipefail
D=gpurun_out/r6i; mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $D/gputests.log 2>&1; rc=$?
tail -25 $D/gputests.log
[ $rc -ne 0 ] && exit 1
KT_LIBS="old:var/libold.so lpc:" bash tools/ktrace_ab.sh $D/kt k_tables || exit 1
AB_LIBS="old:var/libold.so lpc:" AB_REPS=2 bash tools/ab.sh $D/ab3 || exit 1
AB_LIBS="old:var/libold.so lpc:" AB_ARGS="--config 3 --shard-of 8" AB_REPS=2 bash tools/ab.sh $D/s8 || exit 1
