#!/bin/bash
# A/B bench lines for a config under context options: tools/ab_cfg.sh OUTDIR CONFIG REPS "OPTS_A" "OPTS_B" ...
# each OPTS is a space-separated list of NAME=VALUE (or "-" for the product settings)
out=$1; cfg=$2; reps=$3; shift 3
mkdir -p $out
for rep in $(seq 1 $reps); do
  i=0
  for opts in "$@"; do
    i=$((i + 1))
    args=""
    if [ "$opts" != "-" ]; then for o in $opts; do args="$args --opt $o"; done; fi
    timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 $args \
      > $out/c${cfg}_${i}_$rep.json 2> $out/c${cfg}_${i}_$rep.err || { tail -5 $out/c${cfg}_${i}_$rep.err; exit 1; }
    python - "$out/c${cfg}_${i}_$rep.json" "$opts" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("[" + sys.argv[2] + "]", "ms/step", round(d["ms_per_step"], 3), "dev", round(d["device_resident_ms_per_step"], 3),
      "boot launch ms", round(r["avg_launch_ms"], 3), "frac", round(r["frac"], 3),
      "kms", {k: round(v, 3) for k, v in d["kernel_ms_per_step"].items()},
      "piece wait/host", round(d["host_syncs"].get("piece_wait_ms_per_step", 0), 3), round(d["host_syncs"].get("piece_host_ms_per_step", 0), 3))
PY
  done
done
