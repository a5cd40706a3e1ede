#!/bin/bash
set -o pipefail
D=gpurun_out/r6b; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_skip.py -x -q --timeout 250 --timeout-method thread > $D/skip.log 2>&1 || { tail -30 $D/skip.log; exit 1; }
tail -1 $D/skip.log
AB_LIBS="old:var/libold.so lean:  g0:var/libg0.so g0w4:var/libg0w4.so" AB_REPS=2 bash tools/ab.sh $D/ab
