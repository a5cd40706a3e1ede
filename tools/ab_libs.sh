#!/bin/bash
# Config-3 bench lines of the product library against study builds: tools/ab_libs.sh OUTDIR REPS NAME...
# (NAME: diag/libNAME.so from tools/build_variant.sh; "prod" = scde_amd/libscde_hip.so)
out=$1; reps=$2; shift 2
mkdir -p $out
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    lib=""; [ "$v" != prod ] && lib=diag/lib$v.so
    SCDE_LIB=$lib timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 \
      > $out/${v}_$rep.json 2> $out/${v}_$rep.err || { tail -3 $out/${v}_$rep.err; exit 1; }
    python - $out/${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms/step", round(d["ms_per_step"], 3), "dev", round(d["device_resident_ms_per_step"], 3),
      "kms", {k: round(v, 3) for k, v in d["kernel_ms_per_step"].items()})
PY
  done
done
