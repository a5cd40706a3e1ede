#!/bin/bash
# round 5 final measurement, part A: GPU suite, rocprofv3 profiles (stats + PMC passes) of configs 3, 2, 2b, 4
set -o pipefail
mkdir -p gpurun_out/fin5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/fin5/gputests.log 2>&1 || { tail -30 gpurun_out/fin5/gputests.log; exit 1; }
tail -1 gpurun_out/fin5/gputests.log
for c in ${PROF_CFGS:-3 2 2b 4}; do
  PROFILE_PREFIX=profiles/r05_config$c timeout -k 10 900 bash tools/profile.sh gpurun_out/fin5/prof$c --config $c --steps 3 --warmup 1 --cpu-sample 0 --no-profile --opt lanes=1 --opt modes_overlap=0 > gpurun_out/fin5/prof$c.log 2>&1 || { tail -5 gpurun_out/fin5/prof$c.log; exit 1; }
  echo "profiled config $c"
  cp profiles/r05_config${c}_* gpurun_out/fin5/
done
echo done
