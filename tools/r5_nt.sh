#!/bin/bash
# A/B: k_tables_reg rows as non-temporal stores (diag/libnt.so) against the product build, config 3
set -o pipefail
out=gpurun_out/nt; mkdir -p $out
for rep in 1 2 3; do
  for v in nt prod; do
    lib=""; [ $v != prod ] && lib=diag/lib$v.so
    SCDE_LIB=$lib timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 \
      > $out/$v$rep.json 2> $out/$v$rep.err || { tail -3 $out/$v$rep.err; exit 1; }
    python - $out/$v$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms_per_step"]
print(sys.argv[2], "ms/step", round(d["ms_per_step"], 3), "tables", round(k["tables"], 3), "boot", round(k.get("bootstrap", 0), 3))
PY
  done
done
