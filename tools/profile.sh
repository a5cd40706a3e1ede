#!/bin/bash
# rocprofv3 passes over a short bench run (run on the GPU box via gpurun).
#   tools/profile.sh <outdir> [bench args...]
# pass 0: kernel trace + stats; passes 1-5: PMC counters (each in its own run, no trace domains).
set -e
OUT=${1:-gpurun_out/prof}; shift || true
ARGS=${@:-"--steps 3 --warmup 1 --cpu-sample 0 --no-profile --opt lanes=1"}
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d $OUT/pmc1 -o run -- python3 bench.py $ARGS > $OUT/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc2 -o run -- python3 bench.py $ARGS > $OUT/pmc2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD TCC_HIT_sum --output-format csv -d $OUT/pmc3 -o run -- python3 bench.py $ARGS > $OUT/pmc3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/pmc5 -o run -- python3 bench.py $ARGS > $OUT/pmc5.log 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum WRITE_SIZE --output-format csv -d $OUT/pmc4 -o run -- python3 bench.py $ARGS > $OUT/pmc4.log 2>&1
# summary -> profiles/ (PROFILE_PREFIX, e.g. profiles/r01)
[ -n "$PROFILE_PREFIX" ] && python3 tools/pmc_summary.py $OUT $PROFILE_PREFIX
echo profile done
