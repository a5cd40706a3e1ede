#!/bin/bash
# tables_nt: the skip-mode test (both store kinds), then config 2 / 3 with the default (auto) against the other kind
set -o pipefail
out=gpurun_out/nt3; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_skip.py > $out/skip.log 2>&1 || { tail -30 $out/skip.log; exit 1; }
tail -1 $out/skip.log
run() {  # config tag opts...
  c=$1; t=$2; shift 2
  timeout -k 10 200 python bench.py --config $c --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 "$@" \
    > $out/$c$t.json 2> $out/$c$t.err || { tail -3 $out/$c$t.err; return 1; }
  python - $out/$c$t.json $c $t <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms_per_step"]
print(sys.argv[2], sys.argv[3], "ms/step", round(d["ms_per_step"], 3), "dev", round(d["device_resident_ms_per_step"], 3), "tables", round(k["tables"], 3), "boot", round(k["boot"], 3))
PY
}
for rep in 1 2; do
  run 2 auto$rep || exit 1
  run 2 nt$rep --opt tables_nt=1 || exit 1
  run 3 auto$rep || exit 1
  run 3 plain$rep --opt tables_nt=0 || exit 1
done
