# A/B of the host-count upload pipelining threshold (option pipeline_mb) at small matrices
for pm in 0 48; do
for a in "--config 3 --shard-of 8" "--config 3 --shard-of 4" "--config 2"; do
timeout -k 10 200 python bench.py $a --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 --no-profile --opt pipeline_mb=$pm > gpurun_out/pp.log 2>&1 || exit 1
echo "pipeline_mb=$pm $a: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pp.log)"
done; done
