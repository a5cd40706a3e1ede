# pieces / pipelining A/B (GPU box): parity tests first, then host->host ms per step
timeout -k 10 300 python -u -m pytest tests/test_gpu_skip.py tests/test_gpu_configs.py tests/test_gpu_fullsize.py::test_config4_1000_gene_slice_modes -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; rc=$?; tail -3 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for o in "pieces=1" "pieces=2" "pieces=4" "pieces=8"; do
timeout -k 10 200 python bench.py --config 3 --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --no-profile --opt $o > gpurun_out/pc.log 2>&1 || exit 1
echo "config 3 $o: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pc.log | tr '\n' ' ')"
done
for pm in 0 48; do for a in "--config 3 --shard-of 8" "--config 3 --shard-of 4" "--config 2"; do
timeout -k 10 200 python bench.py $a --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --no-profile --opt pipeline_mb=$pm > gpurun_out/pc.log 2>&1 || exit 1
echo "pipeline_mb=$pm $a: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pc.log | tr '\n' ' ')"
done; done
for o in "pieces=1" "pieces=4" "pieces=8"; do
timeout -k 10 200 python bench.py --config 4 --steps 5 --warmup 2 --cpu-sample 0 --cpu-workers 0 --no-profile --opt $o > gpurun_out/pc.log 2>&1 || exit 1
echo "config 4 $o: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pc.log | tr '\n' ' ')"
done
