#!/bin/bash
# round 5, first GPU session: GPU suite, config-3 profile with the FP64 instruction-counter pass,
# config-3 bench line (reads the new profile) and the shard-of-8 projection
set -o pipefail
mkdir -p gpurun_out/r5a
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5a/gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r5a/gputests.log; [ $rc -eq 0 ] || exit $rc
PROFILE_PREFIX=profiles/r05_config3 timeout -k 10 600 bash tools/profile.sh gpurun_out/r5a/prof3 --config 3 --steps 3 --warmup 1 --cpu-sample 0 --no-profile --opt lanes=1 --opt modes_overlap=0 > gpurun_out/r5a/prof3.log 2>&1 || { tail -5 gpurun_out/r5a/prof3.log; exit 1; }
cp profiles/r05_config3_* gpurun_out/r5a/
timeout -k 10 300 python bench.py --config 3 --cpu-sample 0 --cpu-workers 0 > gpurun_out/r5a/b3.json 2> gpurun_out/r5a/b3.err || { tail -5 gpurun_out/r5a/b3.err; exit 1; }
timeout -k 10 200 python bench.py --config 3 --shard-of 8 --cpu-sample 0 --cpu-workers 0 > gpurun_out/r5a/b3s8.json 2> gpurun_out/r5a/b3s8.err || exit 1
grep -o '"ms_per_step": [0-9.e+]*\|device_resident_ms_per_step": [0-9.e+]*' gpurun_out/r5a/b3.json gpurun_out/r5a/b3s8.json
echo done
