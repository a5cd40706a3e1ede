#!/bin/bash
# ELL block size A/B: 16 (default) vs 4 / 8 waves per 64-gene block
set -o pipefail
OUT=gpurun_out/r5z
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 30 --warmup 5 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), {a: round(b,3) for a,b in d.get('kernel_ms_per_step',{}).items()})"
}
for i in 1 2; do
  run c3_$i --config 3
  SCDE_LIB=diag/libell4.so run c3_e4_$i --config 3
  SCDE_LIB=diag/libell8.so run c3_e8_$i --config 3
done
run s8 --config 3 --shard-of 8
SCDE_LIB=diag/libell4.so run s8_e4 --config 3 --shard-of 8
SCDE_LIB=diag/libell8.so run s8_e8 --config 3 --shard-of 8
