#!/bin/bash
# round-6 baseline on the GPU box: GPU suite, smoke, config-3 bench, shard-of-8 bench
set -o pipefail
D=gpurun_out/${R6_DIR:-r6a}
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $D/gputests.log 2>&1 || { tail -30 $D/gputests.log; exit 1; }
tail -1 $D/gputests.log
timeout -k 10 200 python bench.py --config 3 > $D/b_3.json 2> $D/b_3.err || { tail -5 $D/b_3.err; exit 1; }
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*\|device_resident_ms_per_step": [0-9.e+]*\|"frac": [0-9.e+]*' $D/b_3.json | tr '\n' ' '; echo
timeout -k 10 200 python bench.py --config 3 --shard-of 8 --cpu-sample 0 --cpu-workers 0 > $D/b_3_s8.json 2> $D/b_3_s8.err || { tail -5 $D/b_3_s8.err; exit 1; }
grep -o '"ms_per_step": [0-9.e+]*\|device_resident_ms_per_step": [0-9.e+]*' $D/b_3_s8.json | tr '\n' ' '; echo
