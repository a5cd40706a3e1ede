#!/bin/bash
# tile-order keys: count sums (default build) vs count-rank sums (diag/libkeyrank.so):
# FETCH_SIZE of the bootstrap at configs 4 and 3 (lanes 1, read-backs not overlapped), then bench lines
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5o
mkdir -p $OUT
A="--steps 3 --warmup 1 --cpu-sample 0 --cpu-workers 0 --no-profile --opt lanes=1 --opt modes_overlap=0"
for c in 4 3; do
  for v in count rank; do
    if [ $v = rank ]; then export SCDE_LIB=diag/libkeyrank.so; else unset SCDE_LIB; fi
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p${c}_$v -o run -- python3 bench.py --config $c $A > $OUT/p${c}_$v.log 2>&1 || exit 1
    python3 - <<PY
import pandas as pd
d=pd.read_csv('$OUT/p${c}_$v/run_counter_collection.csv')
d=d[d['Kernel_Name'].str.contains('k_boot_gene')]
print('config $c $v k_boot_gene FETCH GB per launch %.2f' % (d['Counter_Value'].mean()*2*1024/1e9))
PY
  done
done
unset SCDE_LIB
run() {
  tag=$1; shift
  timeout -k 10 400 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 20 --warmup 3 "$@" > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), {a: round(b,3) for a,b in d.get('kernel_ms_per_step',{}).items()})"
}
run c4 --config 4
SCDE_LIB=diag/libkeyrank.so run c4r --config 4
run c3 --config 3
SCDE_LIB=diag/libkeyrank.so run c3r --config 3
