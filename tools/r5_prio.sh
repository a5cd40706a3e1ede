#!/bin/bash
# shard of 8 and config 3: peer-lane priority and k_boot_gene launch chunks against the defaults
set -o pipefail
out=gpurun_out/prio; mkdir -p $out
run() {  # tag bench-args...
  t=$1; shift
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 "$@" \
    > $out/$t.json 2> $out/$t.err || { tail -3 $out/$t.err; return 1; }
  python - $out/$t.json $t <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms/step", round(d["ms_per_step"], 3), "dev", round(d["device_resident_ms_per_step"], 3))
PY
}
for rep in 1 2; do
  for v in "def" "prio:--opt lane_prio=1" "ch2:--opt boot_chunks=2" "ch4:--opt boot_chunks=4" "prioch2:--opt lane_prio=1 --opt boot_chunks=2"; do
    t=${v%%:*}; a=""; [ "$v" != "$t" ] && a=${v#*:}
    run s8_$t$rep --config 3 --shard-of 8 $a || exit 1
  done
done
for rep in 1 2; do
  for v in "def" "prio:--opt lane_prio=1" "ch2:--opt boot_chunks=2"; do
    t=${v%%:*}; a=""; [ "$v" != "$t" ] && a=${v#*:}
    run c3_$t$rep --config 3 $a || exit 1
  done
done
