#!/bin/bash
# round 5 closing measurement on the final build: config-3 profile, then the config-3 line and its shards
set -o pipefail
mkdir -p gpurun_out/fin5
PROFILE_PREFIX=profiles/r05_config3 timeout -k 10 900 bash tools/profile.sh gpurun_out/fin5/prof3 --config 3 --steps 3 --warmup 1 --cpu-sample 0 --no-profile --opt lanes=1 --opt modes_overlap=0 > gpurun_out/fin5/prof3.log 2>&1 || { tail -5 gpurun_out/fin5/prof3.log; exit 1; }
cp profiles/r05_config3_* gpurun_out/fin5/
CFGS="3" PROF_CFGS=" " bash tools/r5_final_b.sh || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dist.py -m gpu > gpurun_out/fin5/dist.log 2>&1 || { tail -30 gpurun_out/fin5/dist.log; exit 1; }
tail -3 gpurun_out/fin5/dist.log
timeout -k 10 700 bash tools/r5_nt.sh || exit 1
