timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; rc=$?; tail -4 gpurun_out/gputests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --config 2 --steps 10 --warmup 2 --cpu-sample 0 --cpu-workers 0 > gpurun_out/bc2.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config 3 --steps 5 --warmup 1 --cpu-sample 0 --cpu-workers 0 > gpurun_out/bc3.log 2>&1 || exit 1
grep -ho "\"value\": [0-9.]*\|\"kernel_ms_per_step\": {[^}]*}" gpurun_out/bc2.log gpurun_out/bc3.log
