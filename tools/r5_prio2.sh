#!/bin/bash
# per-call lane priority (lane_prio 2, the default): skip-mode test, A/B against lane_prio 0, then the GPU suite
set -o pipefail
out=gpurun_out/prio2; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_skip.py > $out/skip.log 2>&1 || { tail -30 $out/skip.log; exit 1; }
tail -1 $out/skip.log
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
  run s8_auto$rep --config 3 --shard-of 8 || exit 1
  run s8_off$rep --config 3 --shard-of 8 --opt lane_prio=0 || exit 1
  run c3_auto$rep --config 3 || exit 1
  run c3_off$rep --config 3 --opt lane_prio=0 || exit 1
done
run s4_auto --config 3 --shard-of 4 || exit 1
run s4_off --config 3 --shard-of 4 --opt lane_prio=0 || exit 1
bash tools/r5_check.sh
