# batch DE on two lanes: parity + bit-identity test, then config 2b host->host by lanes (GPU box)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "batch" -x -q --timeout 200 --timeout-method thread > gpurun_out/bt.log 2>&1; rc=$?; tail -3 gpurun_out/bt.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for o in 1 2; do
timeout -k 10 200 python bench.py --config 2b --steps 30 --warmup 5 --cpu-sample 0 --cpu-workers 0 --no-profile --opt lanes=$o > gpurun_out/pb.log 2>&1 || exit 1
echo "config 2b lanes=$o: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pb.log | tr '\n' ' ')"
done; done
