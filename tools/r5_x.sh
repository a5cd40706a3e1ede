#!/bin/bash
# AVX2 narrowing: config 4 host steps (u16 issuer waits), three runs, and the 16-bit upload test
set -o pipefail
OUT=gpurun_out/r5x
mkdir -p $OUT
grep -o -m1 'avx2' /proc/cpuinfo || echo "no avx2"
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 30 --warmup 5 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json')); h=d['host_syncs']
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), 'pw %.3f' % h['piece_wait_ms_per_step'], h['u16_ms_per_step'])"
}
run c4_1 --config 4
run c4_32 --config 4 --opt upload_u16=0
run c4_2 --config 4
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -k "16bit or config4" -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
