#!/bin/bash
# A/B of library builds and/or options on one GPU box (alternating runs):
#   AB_LIBS="old:var/libold.so new: nogate::boot_gate=0" AB_ARGS="--config 3" AB_REPS=2 bash tools/ab.sh OUTDIR
# spec = name:lib[:opt=v,opt=v]; an empty lib = the in-tree build.  Prints host->host,
# device-resident and the per-stage kernel ms per step of each run.
set -o pipefail
out=${1:-gpurun_out/ab}
mkdir -p $out
for r in $(seq 1 ${AB_REPS:-2}); do
  for spec in $AB_LIBS; do
    IFS=: read -r name lib opts <<< "$spec"
    oargs=""
    for o in ${opts//,/ }; do oargs="$oargs --opt $o"; done
    SCDE_LIB=$lib timeout -k 10 300 python bench.py ${AB_ARGS:---config 3} $oargs --steps ${AB_STEPS:-20} --warmup 3 \
      --cpu-sample 0 --cpu-workers 0 > $out/${name}_$r.json 2> $out/${name}_$r.err || { tail -5 $out/${name}_$r.err; exit 1; }
    python - $out/${name}_$r.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {a: round(b, 3) for a, b in d.get("kernel_ms_per_step", {}).items()}
print(f"{sys.argv[2]:10s} host {d['ms_per_step']:.3f} dev {d.get('device_resident_ms_per_step', float('nan')):.3f} {k}")
PY
  done
done
