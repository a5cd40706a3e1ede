#!/bin/bash
# A/B per config: non-temporal table stores (the product build) against plain stores (diag/libplain.so)
set -o pipefail
out=gpurun_out/nt2; mkdir -p $out
for c in 2 4 2b 3; do
  for rep in 1 2; do
    for v in plain nt; do
      lib=""; [ $v != nt ] && lib=diag/lib$v.so
      SCDE_LIB=$lib timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 \
        > $out/$c$v$rep.json 2> $out/$c$v$rep.err || { tail -3 $out/$c$v$rep.err; exit 1; }
      python - $out/$c$v$rep.json $c $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms_per_step"]
print(sys.argv[2], sys.argv[3], "ms/step", round(d["ms_per_step"], 3), "dev", round(d["device_resident_ms_per_step"], 3), "tables", round(k["tables"], 3), "boot", round(k["boot"], 3))
PY
    done
  done
done
