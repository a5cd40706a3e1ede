#!/bin/bash
# shard-of-8 step timelines (host -> host step and device-resident step), default options
set -o pipefail
mkdir -p gpurun_out/r5c
bash tools/tl_shard.sh gpurun_out/r5c/s8h 8 --trace-host || exit 1
cp gpurun_out/r5c/s8h/timeline.txt gpurun_out/r5c/s8_host_timeline.txt
bash tools/tl_shard.sh gpurun_out/r5c/s8d 8 || exit 1
cp gpurun_out/r5c/s8d/timeline.txt gpurun_out/r5c/s8_dev_timeline.txt
rm -rf gpurun_out/r5c/s8h/tl gpurun_out/r5c/s8d/tl
