#!/bin/bash
# config 4: host -> host and device-resident step timelines, and a bench line
set -o pipefail
mkdir -p gpurun_out/r5e
bash tools/tl_cfg.sh gpurun_out/r5e/c4h 4 --trace-host || exit 1
bash tools/tl_cfg.sh gpurun_out/r5e/c4d 4 || exit 1
timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --cpu-sample 0 --cpu-workers 0 \
  > gpurun_out/r5e/b4.json 2> gpurun_out/r5e/b4.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/r5e/b4.json'))
print('host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']), d['kernel_ms_per_step'], d['host_syncs'])"
