# config 3 host->host by piece count, alternating, longer runs (GPU box)
for rep in 1 2; do for o in 1 2 3 4; do
timeout -k 10 200 python bench.py --config 3 --steps 60 --warmup 5 --cpu-sample 0 --cpu-workers 0 --no-profile --opt pieces=$o > gpurun_out/pc.log 2>&1 || exit 1
echo "config 3 pieces=$o: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pc.log | tr '\n' ' ')"
done; done
