#!/bin/bash
# one PMC pass per library build and/or option set; per-kernel mean counters of the kernels matching a
# regex, and their dispatch count and summed duration per bench call:
#   PMC_LIBS="old:var/libold.so new: c1::jp_chunks=1" PMC="SQ_WAVES SQ_INSTS_VALU" bash tools/pmc_ab.sh OUTDIR REGEX
# spec = name:lib[:opt=v,opt=v] as in tools/ab.sh (an empty lib = the in-tree build)
set -o pipefail
out=${1:-gpurun_out/pmc}; re=${2:-k_tables_lpc}
export TMPDIR=/tmp
mkdir -p $out
for spec in $PMC_LIBS; do
  IFS=: read -r name lib opts <<< "$spec"
  oargs=""
  for o in ${opts//,/ }; do oargs="$oargs --opt $o"; done
  SCDE_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc $PMC --output-format csv -d $out/$name -o run -- \
    python3 bench.py ${PMC_ARGS:---config 3 --opt lanes=1} $oargs --steps 3 --warmup 1 --cpu-sample 0 --cpu-workers 0 \
    --no-profile > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }
  f=$(find $out/$name -name "run_counter_collection.csv" | head -1)
  python3 - "$f" "$name" "$re" <<'PY'
import sys
import pandas as pd
d = pd.read_csv(sys.argv[1])
d = d[d["Kernel_Name"].str.contains(sys.argv[3])]
m = d.groupby("Counter_Name")["Counter_Value"].mean()
one = d.drop_duplicates("Dispatch_Id")
calls = 8  # bench --steps 3 --warmup 1 --no-profile: 4 host-count calls + 4 device-resident calls
ms = ((one.End_Timestamp - one.Start_Timestamp) / 1e6).sum() / calls
print(sys.argv[2], f"dispatches/call {len(one) / calls:.2f} ms/call {ms:.3f}", " ".join(f"{k}={v:.4g}" for k, v in m.items()))
PY
done
