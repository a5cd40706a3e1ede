#!/bin/bash
# Quick GPU iteration: bit-identity/oracle tests for the bootstrap kernels, then config-3
# (and optionally more) bench lines.  Usage: tools/quick_check.sh OUTDIR [bench configs...]
out=${1:-gpurun_out/q}; shift
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_skip.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py -x -q \
  --timeout 180 --timeout-method thread > $out/tests.log 2>&1; rc=$?; tail -3 $out/tests.log; [ $rc -eq 0 ] || exit $rc
for c in ${@:-3}; do
  timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 2 --cpu-sample 0 --cpu-workers 0 > $out/bc$c.log 2>&1 || exit 1
  python - "$out/bc$c.log" <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    if ln.startswith("{"):
        d = json.loads(ln)
        r = d.get("roofline", {})
        print(sys.argv[1], "value", round(d["value"]), "ms/step", round(d["ms_per_step"], 3), "dev", d.get("device_resident_genes_per_s"),
              "frac", r.get("frac"), "kms", {k: round(v, 3) for k, v in d.get("kernel_ms_per_step", {}).items()})
PY
done
