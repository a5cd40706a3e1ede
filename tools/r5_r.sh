#!/bin/bash
# config 3 host path: 16-bit uploads x pieces
set -o pipefail
OUT=gpurun_out/r5r
mkdir -p $OUT
show() {
python3 - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); h = d['host_syncs']
print(sys.argv[2], 'host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']),
      'pw %.3f ph %.3f' % (h['piece_wait_ms_per_step'], h['piece_host_ms_per_step']), h.get('u16_ms_per_step'), h['host_phase_ms_per_step'])
PY
}
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 30 --warmup 5 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  show $OUT/b_$tag.json $tag
}
run base --config 3
run u_p4 --config 3 --opt upload_u16=2
run u_p2 --config 3 --opt upload_u16=2 --opt pieces=2
run u_p3 --config 3 --opt upload_u16=2 --opt pieces=3
run base2 --config 3
run p2 --config 3 --opt pieces=2
