#!/bin/bash
# fused two-group posteriors: GPU suite, then config 3 / shard of 8 / config 2 fused vs unfused on one box
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5b/gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r5b/gputests.log; [ $rc -eq 0 ] || exit $rc
for opt in 1 0; do
  for a in "--config 3" "--config 3 --shard-of 8" "--config 2"; do
    tag=$(echo "$a" | tr -d ' -')_f$opt
    timeout -k 10 300 python bench.py $a --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --opt fuse_groups=$opt > gpurun_out/r5b/b_$tag.json 2> gpurun_out/r5b/b_$tag.err || { tail -5 gpurun_out/r5b/b_$tag.err; exit 1; }
    echo "$tag $(grep -o '"ms_per_step": [0-9.e+]*\|device_resident_ms_per_step": [0-9.e+]*' gpurun_out/r5b/b_$tag.json | tr '\n' ' ')"
  done
done
echo done
