#!/bin/bash
# ELL builder A/B: cell chunks by size (default) vs one pass (ell_chunks 1)
set -o pipefail
OUT=gpurun_out/r5n
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 400 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 20 --warmup 3 "$@" \
    > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), {a: round(b,3) for a,b in d.get('kernel_ms_per_step',{}).items()})"
}
for c in 2 2b 3; do
  run c${c} --config $c
  run c${c}_e1 --config $c --opt ell_chunks=1
done
run s8 --config 3 --shard-of 8
run s8_e1 --config 3 --shard-of 8 --opt ell_chunks=1
run c4 --config 4
run c4_e1 --config 4 --opt ell_chunks=1
