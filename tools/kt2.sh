#!/bin/bash
export TMPDIR=/tmp
o=gpurun_out/kt2
mkdir -p $o
for v in 100 200; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $o/t$v -o run -- python3 bench.py --config 2 --steps 3 --warmup 1 --cpu-sample 0 --cpu-workers 0 --no-profile --opt lanes=1 --opt boot_tiles_cells=$v --opt skip_stats=1 > $o/t$v.log 2>&1 || exit 1
done
