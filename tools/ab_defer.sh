# deferred first-group bootstrap (pipelined two-lane DE): tests, then host->host A/B (GPU box)
timeout -k 10 300 python -u -m pytest tests/test_gpu_skip.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dt.log 2>&1; rc=$?; tail -3 gpurun_out/dt.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for o in 1 0; do for c in "--config 3" "--config 3 --shard-of 2"; do
timeout -k 10 200 python bench.py $c --steps 30 --warmup 5 --cpu-sample 0 --cpu-workers 0 --no-profile --opt defer_boot=$o > gpurun_out/pd.log 2>&1 || exit 1
echo "$c defer_boot=$o: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pd.log | tr '\n' ' ')"
done; done; done
