#!/bin/bash
set -o pipefail
D=gpurun_out/r6o; mkdir -p $D
SCDE_LIB=var/libnanpad.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $D/nan.log 2>&1; echo "nanpad suite rc=$?"; tail -3 $D/nan.log
KT_LIBS="cur: nanpad:var/libnanpad.so" bash tools/ktrace_ab.sh $D/kt k_tables_lpc || exit 1
