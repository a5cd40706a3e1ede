#!/bin/bash
# Step timeline of one config at N = 1 (one process, GPU box):
#   tools/tl_cfg.sh OUTDIR CONFIG [extra bench args, e.g. --trace-host]
OUT=$1; CFG=$2; shift 2
export TMPDIR=/tmp
mkdir -p $OUT
timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/tl -o run -- \
  python3 bench.py --config $CFG --steps 3 --warmup 1 --cpu-sample 0 --cpu-workers 0 --no-profile "$@" \
  > $OUT/tl.log 2>&1 || { tail -5 $OUT/tl.log; exit 1; }
python3 tools/timeline.py $OUT/tl > $OUT/timeline.txt && tail -3 $OUT/timeline.txt
rm -rf $OUT/tl
