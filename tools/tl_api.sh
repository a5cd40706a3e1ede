#!/bin/bash
# Step timeline with host API calls (syncs, copies and their threads) of config 3, rank 0's shard
# of an N-way split (N = 1: the whole workload), host-count steps: tools/tl_api.sh OUTDIR N [bench args]
OUT=$1; N=$2; shift 2
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $OUT/tl -o run -- \
  python3 bench.py --config 3 --shard-of $N --steps 3 --warmup 1 --cpu-sample 0 --cpu-workers 0 --no-profile --trace-host "$@" \
  > $OUT/tl.log 2>&1 || { tail -5 $OUT/tl.log; exit 1; }
python3 tools/timeline.py $OUT/tl > $OUT/timeline.txt && tail -3 $OUT/timeline.txt
