#!/bin/bash
# k_boot_gene epilogue timing builds (diag/libe*.so, results wrong by construction): config 3 bootstrap per step
set -o pipefail
OUT=gpurun_out/r5t
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 20 --warmup 3 --config 3 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), {a: round(b,3) for a,b in d.get('kernel_ms_per_step',{}).items()})"
}
run base
for v in 1024 3072 4096 8192; do SCDE_LIB=diag/libe$v.so run e$v; done
run base2
