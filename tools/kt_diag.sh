#!/bin/bash
# k_tables_reg timing builds (diag/libkt*.so from tools/build_variant.sh): config-3 tables ms per
# step with parts of the kernel removed (results wrong; timing only).  tools/kt_diag.sh OUTDIR
out=${1:-gpurun_out/ktd}
mkdir -p $out
for v in prod kt16 kt32 kt2 kt8 kt64; do
  lib=""; [ $v != prod ] && lib=diag/lib$v.so
  SCDE_LIB=$lib timeout -k 10 200 python bench.py --config 3 --steps 10 --warmup 2 --cpu-sample 0 --cpu-workers 0 \
    > $out/$v.json 2> $out/$v.err || { tail -3 $out/$v.err; exit 1; }
  python - $out/$v.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "tables ms/step", round(d["kernel_ms_per_step"]["tables"], 3))
PY
done
