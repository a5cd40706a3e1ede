# persistent upload thread + peer lane priority: tests, then host->host A/B (GPU box)
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wt.log 2>&1; rc=$?; tail -3 gpurun_out/wt.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for o in "lane_prio=1" "lane_prio=0"; do for c in "--config 3" "--config 3 --shard-of 8"; do
timeout -k 10 200 python bench.py $c --steps 30 --warmup 5 --cpu-sample 0 --cpu-workers 0 --no-profile --opt $o > gpurun_out/pw.log 2>&1 || exit 1
echo "$c $o: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pw.log | tr '\n' ' ')"
done; done; done
bash tools/tl_shard.sh gpurun_out/tlw2 1 --trace-host
