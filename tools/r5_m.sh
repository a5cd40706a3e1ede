#!/bin/bash
# config 2 / 2b: tile path at 100 cells per call (boot_tiles_cells 0) against k_boot2; 2b kernel stats
set -o pipefail
OUT=gpurun_out/r5m
mkdir -p $OUT
run() {
  tag=$1; shift
  timeout -k 10 400 python3 bench.py --cpu-sample 0 --cpu-workers 0 --steps 20 --warmup 3 "$@" \
    > $OUT/b_$tag.json 2> $OUT/b_$tag.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/b_$tag.json'))
print('$tag host %.3f dev %s' % (d['ms_per_step'], d.get('device_resident_ms_per_step')), {a: round(b,3) for a,b in d.get('kernel_ms_per_step',{}).items()})"
}
run c2 --config 2
run c2t --config 2 --opt boot_tiles_cells=0
run c2t3 --config 2 --opt boot_tiles_cells=0 --opt gene_waves=3
run c2b --config 2b
run c2bt --config 2b --opt boot_tiles_cells=0
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t2b -o run -- python3 bench.py --config 2b --steps 3 --warmup 1 --cpu-sample 0 --cpu-workers 0 --no-profile --opt lanes=1 > $OUT/t2b.log 2>&1 || exit 1
python3 - <<'PY'
import pandas as pd
d=pd.read_csv('gpurun_out/r5m/t2b/run_kernel_stats.csv')
d['Name']=d['Name'].str.slice(0,60)
print(d[['Name','Calls','AverageNs','TotalDurationNs','Percentage']].head(25).to_string())
PY
