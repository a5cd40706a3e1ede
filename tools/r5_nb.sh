#!/bin/bash
# k_boot2 slab width at config 2 / 2b: boot_nb 20 (default for B = 100) vs 16, 12, 8
set -o pipefail
OUT=gpurun_out/r5nb
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 20 --warmup 3 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %.3f' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), {a: round(b,3) for a,b in d.get('kernel_ms_per_step',{}).items()})"
}
run c2 --config 2
for nb in 16 12 8; do run c2_nb$nb --config 2 --opt boot_nb=$nb; done
run c2b --config 2b
run c2b_nb16 --config 2b --opt boot_nb=16
