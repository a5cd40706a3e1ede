#!/bin/bash
# Gene-block tile bootstrap: bit-identity / oracle tests, then config-3 bench A/B (gene_blocks 1 vs 0).
# Usage: tools/ab_gene.sh OUTDIR
out=${1:-gpurun_out/gene}
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_skip.py tests/test_gpu_fullsize.py tests/test_gpu_configs.py -x -q \
  --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --opt gene_blocks=$v \
    > $out/b3_g$v.json 2> $out/b3_g$v.err || exit 1
  python - "$out/b3_g$v.json" $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("gene_blocks", sys.argv[2], "ms/step", round(d["ms_per_step"], 3), "dev", round(d["device_resident_ms_per_step"], 3),
      "boot launch ms", round(r["avg_launch_ms"], 3), "frac", round(r["frac"], 3), "kms", {k: round(v, 3) for k, v in d["kernel_ms_per_step"].items()})
PY
done
