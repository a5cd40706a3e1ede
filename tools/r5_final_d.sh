#!/bin/bash
# closing config-3 profile on the final build, then its bench line
set -o pipefail
mkdir -p gpurun_out/fin6
PROFILE_PREFIX=profiles/r05_config3 timeout -k 10 900 bash tools/profile.sh gpurun_out/fin6/prof3 --config 3 --steps 3 --warmup 1 --cpu-sample 0 --no-profile --opt lanes=1 --opt modes_overlap=0 > gpurun_out/fin6/prof3.log 2>&1 || { tail -5 gpurun_out/fin6/prof3.log; exit 1; }
cp profiles/r05_config3_* gpurun_out/fin6/
timeout -k 10 400 python bench.py --config 3 > gpurun_out/fin6/b_3.json 2> gpurun_out/fin6/b_3.err || { tail -5 gpurun_out/fin6/b_3.err; exit 1; }
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*\|"frac": [0-9.e+]*' gpurun_out/fin6/b_3.json | tr '\n' ' '
