#!/bin/bash
# shard-of-8 host timelines (tile_order default vs 1), config-4 ELL chunk A/B
set -o pipefail
OUT=gpurun_out/r5h
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --cpu-workers 0 "$@" \
    > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']), {a: round(b,3) for a,b in d['kernel_ms_per_step'].items()}, d['host_syncs'])"
}
run s8 --config 3 --shard-of 8
run s8_o1 --config 3 --shard-of 8 --opt tile_order=1
run c4_e1 --config 4 --opt ell_chunks=1
run c4_e2 --config 4 --opt ell_chunks=2
bash tools/tl_shard.sh $OUT/s8h 8 --trace-host || exit 1
bash tools/tl_shard.sh $OUT/s8h1 8 --trace-host --opt tile_order=1 || exit 1
