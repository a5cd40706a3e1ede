#!/bin/bash
# One part of the end-of-round measurement (GPU box; gpurun limits a call to 20 minutes):
#   tools/measure_part.sh TAG "PROFILED CONFIGS" "BENCH CONFIGS" [tests]
# per profiled config: rocprofv3 stats + PMC passes (tools/profile.sh, lanes = 1) -> profiles/TAG_config<C>_*;
# per bench config: the default bench line -> gpurun_out/fin/b_<C>.json (reads the summary just written)
set -o pipefail
TAG=$1; PROF_CFGS=$2; CFGS=$3; TESTS=$4
mkdir -p gpurun_out/fin
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fin/gputests.log 2>&1 || { tail -20 gpurun_out/fin/gputests.log; exit 1; }
  tail -1 gpurun_out/fin/gputests.log
fi
for c in $PROF_CFGS; do
  PROFILE_PREFIX=profiles/${TAG}_config$c timeout -k 10 600 bash tools/profile.sh gpurun_out/prof${c}_$TAG --config $c --steps 3 --warmup 1 --cpu-sample 0 --no-profile --opt lanes=1 --opt modes_overlap=0 > gpurun_out/fin/prof$c.log 2>&1 || { tail -5 gpurun_out/fin/prof$c.log; exit 1; }
  cp profiles/${TAG}_config${c}_* gpurun_out/fin/
  echo "profiled config $c"
done
for c in $CFGS; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/fin/b_$c.json 2> gpurun_out/fin/b_$c.err || { tail -5 gpurun_out/fin/b_$c.err; exit 1; }
  echo "config $c: $(grep -o '"value": [0-9.e+]*' gpurun_out/fin/b_$c.json) $(grep -o '"ms_per_step": [0-9.e+]*' gpurun_out/fin/b_$c.json)"
done
echo part done
