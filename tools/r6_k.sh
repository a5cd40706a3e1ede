#!/bin/bash
set -o pipefail
D=gpurun_out/r6k; mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_gpu_skip.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread > $D/t.log 2>&1 || { tail -30 $D/t.log; exit 1; }
tail -1 $D/t.log
KT_LIBS="old:var/libold.so lpc: tab:var/libtab.so" bash tools/ktrace_ab.sh $D/kt k_tables_lpc\|k_tables_reg || exit 1
PMC_LIBS="lpc:" PMC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS" bash tools/pmc_ab.sh $D/pmc1 "k_tables_lpc" || exit 1
