#!/bin/bash
# Round-4 GPU check: the whole GPU suite, then config-3 bench lines: product (gene blocks, closed-form
# tables) and the A/B legs (gene_blocks=0; the saddle-point tables build diag/libsaddle.so).
# Usage: tools/r4_check.sh OUTDIR
out=${1:-gpurun_out/r4}
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/gputests.log 2>&1
rc=$?; tail -3 $out/gputests.log; [ $rc -eq 0 ] || exit $rc
line() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "ms/step", round(d["ms_per_step"], 3), "dev", round(d["device_resident_ms_per_step"], 3),
      "boot launch ms", round(r["avg_launch_ms"], 3), "frac", round(r["frac"], 3),
      "kms", {k: round(v, 3) for k, v in d["kernel_ms_per_step"].items()})
PY
}
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 > $out/b3_prod_$rep.json 2> $out/b3_prod_$rep.err || exit 1
  line $out/b3_prod_$rep.json "product"
  timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --opt gene_blocks=0 > $out/b3_slab_$rep.json 2> $out/b3_slab_$rep.err || exit 1
  line $out/b3_slab_$rep.json "gene_blocks=0"
  SCDE_LIB=diag/libsaddle.so timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 > $out/b3_saddle_$rep.json 2> $out/b3_saddle_$rep.err || exit 1
  line $out/b3_saddle_$rep.json "saddle tables"
done
