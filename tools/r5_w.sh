#!/bin/bash
# piece layouts at configs 4 and 3: equal 4 (default), ascending sizes, 8 equal pieces
set -o pipefail
OUT=gpurun_out/r5w
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 30 --warmup 5 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json')); h=d['host_syncs']
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), 'pw %.3f ph %.3f' % (h['piece_wait_ms_per_step'], h['piece_host_ms_per_step']))"
}
for i in 1 2; do
  run c4_$i --config 4
  run c4_asc_$i --config 4 --opt piece_taper=2
  run c4_p8_$i --config 4 --opt pieces=8
  run c3_$i --config 3
  run c3_asc_$i --config 3 --opt piece_taper=2
done
