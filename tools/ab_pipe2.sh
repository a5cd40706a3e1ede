# pipelining threshold at the 2- and 4-way shards (20-40 MB matrices), alternating (GPU box)
for rep in 1 2; do for pm in 0 48; do for n in 2 4; do
timeout -k 10 200 python bench.py --config 3 --shard-of $n --steps 30 --warmup 5 --cpu-sample 0 --cpu-workers 0 --no-profile --opt pipeline_mb=$pm > gpurun_out/pp.log 2>&1 || exit 1
echo "pipeline_mb=$pm shard-of $n: $(grep -o '"ms_per_step": [0-9.]*\|device_resident_ms_per_step": [0-9.]*' gpurun_out/pp.log | tr '\n' ' ')"
done; done; done
