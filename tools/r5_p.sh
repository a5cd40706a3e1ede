#!/bin/bash
# same-box A/B against the round-4 build (oldr04/: a worktree of the r04 commit with its own library):
# configs 3 and 2, alternating, 30 steps each
set -o pipefail
OUT=gpurun_out/r5p
mkdir -p $OUT
run() {
  tag=$1; dir=$2; shift 2
  (cd $dir && timeout -k 10 400 python3 bench.py --cpu-sample 0 --cpu-workers 0 "$@") > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), {a: round(b,3) for a,b in d.get('kernel_ms_per_step',{}).items()})"
}
for i in 1 2; do
  run c3_new$i . --config 3
  run c3_old$i oldr04 --config 3
done
run c2_new . --config 2
run c2_old oldr04 --config 2
run s8_new . --config 3 --shard-of 8
run s8_old oldr04 --config 3 --shard-of 8
