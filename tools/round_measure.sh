#!/bin/bash
# End-of-round measurement on the GPU box (run via gpurun):
#   GPU parity tests, rocprofv3 stats + PMC passes per profiled config (profiles/rNN_config<C>_*),
#   then every bench config with its CPU baseline -> gpurun_out/fin/b_<cfg>.json.
#   tools/round_measure.sh <round tag, e.g. r02> [bench configs...]
#   PROF_CFGS (default: every config) picks the profiled configs; SKIP_TESTS=1 skips the parity tests.
set -o pipefail
TAG=${1:-r02}; shift || true
CFGS=${@:-"3 2 4 2b prior 5"}
PROF_CFGS=${PROF_CFGS:-"2 3 4 2b prior 5"}
mkdir -p gpurun_out/fin
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fin/gputests.log 2>&1 || { tail -20 gpurun_out/fin/gputests.log; exit 1; }
  tail -1 gpurun_out/fin/gputests.log
fi
for c in $PROF_CFGS; do
  PROFILE_PREFIX=profiles/${TAG}_config$c timeout -k 10 1000 bash tools/profile.sh gpurun_out/prof${c}_$TAG --config $c --steps 3 --warmup 1 --cpu-sample 0 --no-profile --opt lanes=1 --opt modes_overlap=0 > gpurun_out/fin/prof$c.log 2>&1 || { tail -5 gpurun_out/fin/prof$c.log; exit 1; }
  echo "profiled config $c"
done
cp profiles/${TAG}_* gpurun_out/fin/ 2>/dev/null
# benches last: each reads its roofline traffic from the summary just written
for c in $CFGS; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/fin/b_$c.json 2> gpurun_out/fin/b_$c.err || { tail -5 gpurun_out/fin/b_$c.err; exit 1; }
  echo "config $c: $(grep -o '"value": [0-9.e+]*' gpurun_out/fin/b_$c.json)"
done
echo measure done
