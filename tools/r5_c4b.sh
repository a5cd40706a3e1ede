#!/bin/bash
# config 4 read-back overlap: tests, then A/B bench lines (jp_chunks) and a host timeline
set -o pipefail
mkdir -p gpurun_out/r5f
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "posteriors or config4" \
  > gpurun_out/r5f/tests.log 2>&1 || { tail -30 gpurun_out/r5f/tests.log; exit 1; }
tail -3 gpurun_out/r5f/tests.log
for ch in 4 2 1; do
  timeout -k 10 300 python3 bench.py --config 4 --steps 10 --warmup 3 --cpu-sample 0 --cpu-workers 0 --opt jp_chunks=$ch \
    > gpurun_out/r5f/b4_$ch.json 2> gpurun_out/r5f/b4_$ch.err || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r5f/b4_$ch.json'))
print('chunks $ch host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']), {a: round(b,3) for a,b in d['kernel_ms_per_step'].items()})"
done
bash tools/tl_cfg.sh gpurun_out/r5f/c4h 4 --trace-host || exit 1
