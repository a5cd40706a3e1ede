#!/bin/bash
# round 5 final measurement, part B: profiles of prior and config 5, then every bench line with its CPU baseline
set -o pipefail
mkdir -p gpurun_out/fin5
for c in ${PROF_CFGS:-prior 5}; do
  PROFILE_PREFIX=profiles/r05_config$c timeout -k 10 900 bash tools/profile.sh gpurun_out/fin5/prof$c --config $c --steps 3 --warmup 1 --cpu-sample 0 --no-profile --opt lanes=1 --opt modes_overlap=0 > gpurun_out/fin5/prof$c.log 2>&1 || { tail -5 gpurun_out/fin5/prof$c.log; exit 1; }
  echo "profiled config $c"
  cp profiles/r05_config${c}_* gpurun_out/fin5/
done
for c in ${CFGS:-3 2 4 2b prior 5}; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/fin5/b_$c.json 2> gpurun_out/fin5/b_$c.err || { tail -5 gpurun_out/fin5/b_$c.err; exit 1; }
  echo "config $c: $(grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*' gpurun_out/fin5/b_$c.json | tr '\n' ' ')"
done
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --config 3 --shard-of $n --cpu-sample 0 --cpu-workers 0 > gpurun_out/fin5/b_3_s$n.json 2> gpurun_out/fin5/b_3_s$n.err || exit 1
  echo "shard of $n: $(grep -o '"ms_per_step": [0-9.e+]*\|device_resident_ms_per_step": [0-9.e+]*' gpurun_out/fin5/b_3_s$n.json | tr '\n' ' ')"
done
echo done
