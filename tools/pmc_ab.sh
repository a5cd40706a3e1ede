#!/bin/bash
# one PMC pass per library build; per-kernel mean counters of the kernels matching a regex:
#   PMC_LIBS="old:var/libold.so new:" PMC="SQ_WAVES SQ_INSTS_VALU" bash tools/pmc_ab.sh OUTDIR REGEX
set -o pipefail
out=${1:-gpurun_out/pmc}; re=${2:-k_tables_lpc}
export TMPDIR=/tmp
mkdir -p $out
for spec in $PMC_LIBS; do
  name=${spec%%:*}; lib=${spec#*:}
  SCDE_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $out/$name -o run -- \
    python3 bench.py ${PMC_ARGS:---config 3 --opt lanes=1} --steps 3 --warmup 1 --cpu-sample 0 --cpu-workers 0 --no-profile \
    > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }
  f=$(find $out/$name -name "run_counter_collection.csv" | head -1)
  python3 - "$f" "$name" "$re" <<'PY'
import sys
import pandas as pd
d = pd.read_csv(sys.argv[1])
d = d[d["Kernel_Name"].str.contains(sys.argv[3])]
m = d.groupby("Counter_Name")["Counter_Value"].mean()
print(sys.argv[2], " ".join(f"{k}={v:.4g}" for k, v in m.items()))
PY
done
