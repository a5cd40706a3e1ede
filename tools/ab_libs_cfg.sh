#!/bin/bash
# Bench lines of study builds across configs: tools/ab_libs_cfg.sh OUTDIR REPS "CFG[:opt=v,...]" ... -- NAME...
# (NAME: diag/libNAME.so from tools/build_variant.sh; "prod" = scde_amd/libscde_hip.so)
out=$1; reps=$2; shift 2
cfgs=()
while [ "$1" != "--" ]; do cfgs+=("$1"); shift; done
shift
mkdir -p $out
for rep in $(seq 1 $reps); do
  for c in "${cfgs[@]}"; do
    cfg=${c%%:*}; opts=""
    [ "$c" != "$cfg" ] && for o in $(echo ${c#*:} | tr ',' ' '); do opts="$opts --opt $o"; done
    for v in "$@"; do
      lib=""; [ "$v" != prod ] && lib=diag/lib$v.so
      f=$out/${v}_c${cfg}_$rep
      SCDE_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 $opts \
        > $f.json 2> $f.err || { tail -3 $f.err; exit 1; }
      python - $f.json "$v $c" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms/step", round(d["ms_per_step"], 3), "dev", round(d["device_resident_ms_per_step"], 3),
      "kms", {k: round(v, 3) for k, v in d["kernel_ms_per_step"].items()})
PY
    done
  done
done
