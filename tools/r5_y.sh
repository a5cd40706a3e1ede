#!/bin/bash
# config 3 with 16-bit uploads in DE calls too (upload_u16 2) vs default, alternating; config 4 line
set -o pipefail
OUT=gpurun_out/r5y
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 30 --warmup 5 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json')); h=d['host_syncs']
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), 'pw %.3f ph %.3f' % (h['piece_wait_ms_per_step'], h['piece_host_ms_per_step']), h['u16_ms_per_step'])"
}
for i in 1 2; do
  run c3_$i --config 3
  run c3u_$i --config 3 --opt upload_u16=2
done
run s8 --config 3 --shard-of 8
run s8u --config 3 --shard-of 8 --opt upload_u16=2
