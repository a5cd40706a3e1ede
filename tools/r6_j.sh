#!/bin/bash
set -o pipefail
D=gpurun_out/r6j; mkdir -p $D
KT_LIBS="lpc: p1:var/libp1.so p2:var/libp2.so p4:var/libp4.so p7:var/libp7.so" bash tools/ktrace_ab.sh $D/kt k_tables_lpc || exit 1
KT_LIBS="lpc_nt0:" KT_ARGS="--config 3 --opt lanes=1 --opt tables_nt=0" bash tools/ktrace_ab.sh $D/kt2 k_tables_lpc || exit 1
PMC_LIBS="old:var/libold.so lpc:" PMC="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS" bash tools/pmc_ab.sh $D/pmc1 "k_tables_reg|k_tables_lpc" || exit 1
PMC_LIBS="old:var/libold.so lpc:" PMC="WRITE_SIZE TCC_EA0_WRREQ_sum" bash tools/pmc_ab.sh $D/pmc2 "k_tables_reg|k_tables_lpc" || exit 1
PMC_LIBS="lpc:" PMC="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH" bash tools/pmc_ab.sh $D/pmc3 "k_tables_lpc" || exit 1
