#!/bin/bash
# GPU suite, then config 4 / config 3 / shard-of-8 bench lines (tile_order 1 vs 2) and a config-4 host timeline
set -o pipefail
OUT=gpurun_out/r5g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/gputests.log 2>&1 || { tail -40 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --cpu-sample 0 --cpu-workers 0 "$@" \
    > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']), {a: round(b,3) for a,b in d['kernel_ms_per_step'].items()})"
}
run c4 --config 4
run c4_o1 --config 4 --opt tile_order=1
run c3 --config 3
run c3_o0 --config 3 --opt tile_order=0
run s8 --config 3 --shard-of 8
run s8_o1 --config 3 --shard-of 8 --opt tile_order=1
bash tools/tl_cfg.sh $OUT/c4h 4 --trace-host || exit 1
