#!/bin/bash
# rest_thread A/B: shard of 8 and config 3 (ms per step host -> host, device-resident)
for o in "" "--opt rest_thread=1" "" "--opt rest_thread=1"; do
  timeout -k 10 200 python bench.py --config 3 --shard-of 8 --cpu-sample 0 --cpu-workers 0 --steps 40 $o > gpurun_out/rt.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/rt.json').read().strip().splitlines()[-1]);print('s8', sys.argv[1:], round(d['ms_per_step'],3), round(d['device_resident_ms_per_step'],3))" $o
done
for o in "" "--opt rest_thread=1"; do
  timeout -k 10 200 python bench.py --config 3 --cpu-sample 0 --cpu-workers 0 --steps 20 $o > gpurun_out/rt3.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/rt3.json').read().strip().splitlines()[-1]);print('c3', sys.argv[1:], round(d['ms_per_step'],3), round(d['device_resident_ms_per_step'],3))" $o
done
