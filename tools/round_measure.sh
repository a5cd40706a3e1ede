#!/bin/bash
# End-of-round measurement on the GPU box (run via gpurun):
#   GPU parity tests, rocprofv3 passes, then every bench config with its CPU baseline -> gpurun_out/fin/b_<cfg>.json,
#   rocprofv3 stats + PMC passes for config 2 (profiles/rNN_*) and config 3 (profiles/rNN_config3_*).
#   tools/round_measure.sh <round tag, e.g. r01> [configs...]
set -o pipefail
TAG=${1:-r01}; shift || true
CFGS=${@:-"2 3 4 2b prior 5"}
mkdir -p gpurun_out/fin
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fin/gputests.log 2>&1 || { tail -20 gpurun_out/fin/gputests.log; exit 1; }
tail -1 gpurun_out/fin/gputests.log
PROFILE_PREFIX=profiles/$TAG timeout -k 10 1000 bash tools/profile.sh gpurun_out/prof_$TAG > gpurun_out/fin/prof2.log 2>&1 || { tail -5 gpurun_out/fin/prof2.log; exit 1; }
PROFILE_PREFIX=profiles/${TAG}_config3 timeout -k 10 1000 bash tools/profile.sh gpurun_out/prof3_$TAG --config 3 --steps 3 --warmup 1 --cpu-sample 0 --no-profile > gpurun_out/fin/prof3.log 2>&1 || { tail -5 gpurun_out/fin/prof3.log; exit 1; }
cp profiles/${TAG}_* gpurun_out/fin/ 2>/dev/null
# benches last: config 2 reads its roofline traffic from the summary just written
for c in $CFGS; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/fin/b_$c.json 2> gpurun_out/fin/b_$c.err || { tail -5 gpurun_out/fin/b_$c.err; exit 1; }
  echo "config $c: $(grep -o '"value": [0-9.e+]*' gpurun_out/fin/b_$c.json)"
done
echo measure done
