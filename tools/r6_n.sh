#!/bin/bash
set -o pipefail
D=gpurun_out/r6n; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_skip.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 1; }
tail -1 $D/t.log
KT_LIBS="tw0: tw1:var/libtw1.so" bash tools/ktrace_ab.sh $D/kt k_tables_lpc || exit 1
PMC_LIBS="tw0: tw1:var/libtw1.so" PMC="WRITE_SIZE TCC_EA0_WRREQ_sum" bash tools/pmc_ab.sh $D/pmc2 "k_tables_lpc" || exit 1
