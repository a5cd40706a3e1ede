#!/bin/bash
# Kernel trace of one tools/qdiag.py run: every kernel's duration in launch order (for per-launch
# questions the slot sums hide).  tools/ktrace.sh OUTDIR CONFIG [option=value ...]
OUT=$1; CFG=$2; shift 2
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 tools/qdiag.py $CFG boot_tiles=1 "$@" > $OUT/kt.log 2>&1 || exit 1
python3 - $OUT <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/kt/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 2 steps' worth of kernels (qdiag ends with 3 timed steps)
with open(sys.argv[1] + "/sequence.txt", "w") as o:
    for r in rows:
        nm = r["Kernel_Name"].split("(")[0].replace("void ", "")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        o.write(f"{int(r['Start_Timestamp'])} {d:10.1f} us  {nm}\n")
PY
grep -E "k_tables_reg|k_boot_tiles|k_ratio|k_boot2_list|k_sum_partials" $OUT/sequence.txt | tail -24
