#!/bin/bash
# upload worker latencies and the 16-bit upload issuer's waits at configs 4 and 3
set -o pipefail
OUT=gpurun_out/r5q
mkdir -p $OUT
show() {
python3 - "$1" "$2" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); h = d['host_syncs']
print(sys.argv[2], 'host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']),
      'wake %.3f first %.3f' % (h['upload_wake_ms_per_step'], h['upload_first_ms_per_step']),
      'pw %.3f ph %.3f' % (h['piece_wait_ms_per_step'], h['piece_host_ms_per_step']), h.get('u16_ms_per_step'))
PY
}
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 20 --warmup 3 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  show $OUT/b_$tag.json $tag
}
run c4 --config 4
run c4_t8 --config 4 --opt upload_threads=8
run c4_32 --config 4 --opt upload_u16=0
run c3u --config 3 --opt upload_u16=2
