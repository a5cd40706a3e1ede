#!/bin/bash
# config 3 host timelines with 16-bit uploads on / off
set -o pipefail
bash tools/tl_cfg.sh gpurun_out/r5k/c3u 3 --trace-host || exit 1
bash tools/tl_cfg.sh gpurun_out/r5k/c3i 3 --trace-host --opt upload_u16=0 || exit 1
