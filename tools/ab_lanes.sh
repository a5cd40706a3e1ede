timeout -k 10 300 python -u -m pytest tests/test_gpu_skip.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lt.log 2>&1; rc=$?; tail -3 gpurun_out/lt.log; [ $rc -eq 0 ] || exit $rc
for o in 2 1; do
timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --opt lanes=$o > gpurun_out/b3_$o.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config 3 --shard-of 8 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --opt lanes=$o > gpurun_out/bs8_$o.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --config 3 --shard-of 4 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --opt lanes=$o > gpurun_out/bs4_$o.log 2>&1 || exit 1
echo lanes=$o; grep -ho "\"ms_per_step\": [0-9.]*\|device_resident_ms_per_step\": [0-9.]*" gpurun_out/b3_$o.log gpurun_out/bs4_$o.log gpurun_out/bs8_$o.log
done
bash tools/tl_shard.sh gpurun_out/tl8l 8
