#!/bin/bash
# GPU suite + bench lines for every config at the current defaults
set -o pipefail
OUT=gpurun_out/r5l
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/gputests.log 2>&1 || { tail -40 $OUT/gputests.log; exit 1; }
tail -2 $OUT/gputests.log
run() {
  tag=$1; shift
  timeout -k 10 400 python3 bench.py --cpu-sample 0 --cpu-workers 0 "$@" \
    > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), {a: round(b,3) for a,b in d.get('kernel_ms_per_step',{}).items()})"
}
run c4 --config 4
run c3 --config 3
run c2 --config 2
run c2b --config 2b
run s8 --config 3 --shard-of 8
run s2 --config 3 --shard-of 2
