#!/bin/bash
# Shard-of-N A/B: tools/ab_shard.sh N REPS "OPTS_A" "OPTS_B" ... (OPTS: space-separated name=value, or "-")
n=$1; reps=$2; shift 2
for rep in $(seq 1 $reps); do
  for opts in "$@"; do
    args=""
    if [ "$opts" != "-" ]; then for o in $opts; do args="$args --opt $o"; done; fi
    timeout -k 10 200 python bench.py --config 3 --shard-of $n --cpu-sample 0 --cpu-workers 0 --steps 40 $args > gpurun_out/abs.json 2>/dev/null || exit 1
    python -c "import json,sys;d=json.loads(open('gpurun_out/abs.json').read().strip().splitlines()[-1]);print('shard', sys.argv[1], sys.argv[2], round(d['ms_per_step'],3), round(d['device_resident_ms_per_step'],3))" $n "[$opts]"
  done
done
