#!/bin/bash
# tapered pieces: A/B (piece_taper 1 vs 0) at configs 3 and 4, alternating; then the pipeline tests
set -o pipefail
OUT=gpurun_out/r5v
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 30 --warmup 5 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json')); h=d['host_syncs']
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), 'pw %.3f ph %.3f' % (h['piece_wait_ms_per_step'], h['piece_host_ms_per_step']))"
}
for i in 1 2; do
  run c3_t1_$i --config 3
  run c3_t0_$i --config 3 --opt piece_taper=0
  run c4_t1_$i --config 4
  run c4_t0_$i --config 4 --opt piece_taper=0
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
