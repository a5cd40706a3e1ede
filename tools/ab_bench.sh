#!/bin/bash
# A/B bench lines for study builds: tools/ab_bench.sh OUTDIR "CONFIGS" LIB... (LIB "main" =
# the in-tree library, "main:NAME=V,NAME2=V2" = it with context options, else diag/libLIB.so).
# Prints value, ms/step and per-stage ms.
out=$1; cfgs=$2; shift 2
mkdir -p $out
for lib in "$@"; do
  for c in $cfgs; do
    opts=""; name=${lib%%:*}
    if [[ "$lib" == *:* ]]; then for o in $(echo ${lib#*:} | tr , ' '); do opts="$opts --opt $o"; done; fi
    if [ "$name" = main ]; then env=""; else env="SCDE_LIB=diag/lib$name.so"; fi
    env $env timeout -k 10 200 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 --cpu-sample 0 --cpu-workers 0 $opts \
      > "$out/$lib.$c.log" 2>&1 || { tail -5 "$out/$lib.$c.log"; exit 1; }
    python - "$out/$lib.$c.log" "$lib" "$c" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        print(f"{sys.argv[2]:>8} cfg {sys.argv[3]}: {d['value']:.0f} {d['ms_per_step']:.3f} ms/step",
              {k: round(v, 3) for k, v in d.get("kernel_ms_per_step", {}).items()})
PY
  done
done
