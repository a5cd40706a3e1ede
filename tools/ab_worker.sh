# upload worker: parity/bit-identity tests, then host->host A/B by piece count and a host-step timeline (GPU box)
timeout -k 10 300 python -u -m pytest tests/test_gpu_skip.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py::test_config4_1000_gene_slice_modes -x -q --timeout 200 --timeout-method thread > gpurun_out/wt.log 2>&1; rc=$?; tail -3 gpurun_out/wt.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for o in 1 2 4 8; do
timeout -k 10 200 python bench.py --config 3 --steps 30 --warmup 5 --cpu-sample 0 --cpu-workers 0 --no-profile --opt pieces=$o > gpurun_out/pw.log 2>&1 || exit 1
echo "config 3 pieces=$o: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pw.log | tr '\n' ' ')"
done; done
for o in 1 4 8; do
timeout -k 10 200 python bench.py --config 4 --steps 10 --warmup 3 --cpu-sample 0 --cpu-workers 0 --no-profile --opt pieces=$o > gpurun_out/pw.log 2>&1 || exit 1
echo "config 4 pieces=$o: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pw.log | tr '\n' ' ')"
done
timeout -k 10 200 python bench.py --config 3 --shard-of 2 --steps 30 --warmup 5 --cpu-sample 0 --cpu-workers 0 --no-profile > gpurun_out/pw.log 2>&1 || exit 1
echo "shard-of 2: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pw.log | tr '\n' ' ')"
bash tools/tl_shard.sh gpurun_out/tlw1 1 --trace-host
