#!/bin/bash
# ELL block size A/B, second round: 16 (default) vs 8 waves, alternating
set -o pipefail
OUT=gpurun_out/r5z2
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 30 --warmup 5 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %.3f' % (d['ms_per_step'], d.get('device_resident_ms_per_step')))"
}
for i in 1 2 3; do
  run s8_$i --config 3 --shard-of 8
  SCDE_LIB=diag/libell8.so run s8_e8_$i --config 3 --shard-of 8
done
for i in 1 2; do
  run c3_$i --config 3
  SCDE_LIB=diag/libell8.so run c3_e8_$i --config 3
  run c4_$i --config 4
  SCDE_LIB=diag/libell8.so run c4_e8_$i --config 4
done
