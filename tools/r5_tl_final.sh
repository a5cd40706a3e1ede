#!/bin/bash
# round 5 step timelines (kernel + memory-copy trace): config 4 host step, config 3 host step,
# rank 0's shard of 8 (device-resident and host steps)
set -o pipefail
bash tools/tl_cfg.sh gpurun_out/r5tl/c4h 4 --trace-host || exit 1
bash tools/tl_cfg.sh gpurun_out/r5tl/c3h 3 --trace-host || exit 1
bash tools/tl_shard.sh gpurun_out/r5tl/s8d 8 || exit 1
rm -rf gpurun_out/r5tl/s8d/tl
bash tools/tl_shard.sh gpurun_out/r5tl/s8h 8 --trace-host || exit 1
rm -rf gpurun_out/r5tl/s8h/tl
