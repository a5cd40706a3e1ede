#!/bin/bash
# per-kernel average durations (rocprofv3 --kernel-trace --stats) of library builds, one pass each:
#   KT_LIBS="old:var/libold.so new:" KT_ARGS="--config 3 --opt lanes=1" bash tools/ktrace_ab.sh OUTDIR [KERNEL_REGEX]
set -o pipefail
out=${1:-gpurun_out/kt}; re=${2:-k_tables|k_boot_gene|k_boot_tiles|k_ratio|k_ell|k_sum}
export TMPDIR=/tmp
mkdir -p $out
for spec in $KT_LIBS; do
  name=${spec%%:*}; lib=${spec#*:}
  SCDE_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$name -o run -- \
    python3 bench.py ${KT_ARGS:---config 3 --opt lanes=1} --steps 5 --warmup 2 --cpu-sample 0 --cpu-workers 0 --no-profile \
    > $out/$name.log 2>&1 || { tail -5 $out/$name.log; exit 1; }
  f=$(find $out/$name -name "run_kernel_stats.csv" | head -1)
  python3 - "$f" "$name" "$re" <<'PY'
import re, sys
import pandas as pd
d = pd.read_csv(sys.argv[1])
d = d[d["Name"].str.contains(sys.argv[3])]
for _, r in d.iterrows():
    n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("scde::", "")
    print(f"{sys.argv[2]:8s} {n:40s} calls {int(r['Calls']):4d} avg_ms {r['AverageNs'] / 1e6:.4f} tot_ms {r['TotalDurationNs'] / 1e6:.3f}")
PY
done
