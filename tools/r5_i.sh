#!/bin/bash
# 16-bit uploads: GPU suite, then A/B bench lines (upload_u16 1 vs 0) for configs 4, 3 and the shard of 8
set -o pipefail
OUT=gpurun_out/r5i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/gputests.log 2>&1 || { tail -40 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 "$@" \
    > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']), {a: round(b,3) for a,b in d['kernel_ms_per_step'].items()}, round(d['host_syncs']['piece_wait_ms_per_step'],3))"
}
run c4 --config 4
run c4_32 --config 4 --opt upload_u16=0
run c3 --config 3
run c3_32 --config 3 --opt upload_u16=0
run s8 --config 3 --shard-of 8
run c4b --config 4
run c4b_32 --config 4 --opt upload_u16=0
