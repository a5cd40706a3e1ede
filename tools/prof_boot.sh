#!/bin/bash
# Focused counters for one kernel over tools/qdiag.py (one config, one option set).
#   tools/prof_boot.sh OUTDIR CONFIG KERNEL_REGEX [option=value ...]
OUT=$1; CFG=$2; KRE=$3; shift 3
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 200 python3 tools/qdiag.py $CFG boot_tiles=1 "$@" > $OUT/qdiag.log 2>&1 || exit 1
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS" \
         "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TD_BUSY_avr TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
         "TCC_HIT_sum TCC_MISS_sum FETCH_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "$KRE" --pmc $P --output-format csv -d $OUT/pmc$i -o run -- python3 tools/qdiag.py $CFG boot_tiles=1 "$@" > $OUT/pmc$i.log 2>&1 || echo "pass $i failed"
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"][:40]
        agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
        n[(k, row["Counter_Name"])] += 1
for k, d in agg.items():
    print(k, {c: f"{v / max(n[(k, c)], 1):.4g}" for c, v in sorted(d.items())})
PY
