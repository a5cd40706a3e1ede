#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5d
run() {
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 > gpurun_out/r5d/b_$tag.json 2> gpurun_out/r5d/b_$tag.err || { tail -5 gpurun_out/r5d/b_$tag.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/r5d/b_$tag.json'))
k=d['kernel_ms_per_step']
print('$tag', 'host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']), 'kern', {a: round(b,3) for a,b in k.items()})"
}
run base --config 3
for d in 528 16 144 272; do SCDE_LIB=diag/libt$d.so run diag$d --config 3; done
