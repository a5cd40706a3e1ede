# round measurement, part A (GPU box): GPU tests, config 3 profile + bench, shard projections, timelines
bash tools/measure_part.sh r03 "3" "3" tests || exit 1
for n in 2 4 8; do
timeout -k 10 200 python bench.py --config 3 --shard-of $n --cpu-sample 0 --cpu-workers 0 > gpurun_out/fin/b_3_shard_of_$n.json 2> gpurun_out/fin/b_3_shard_$n.err || exit 1
echo "shard-of $n: $(grep -o '"ms_per_step": [0-9.e+]*' gpurun_out/fin/b_3_shard_of_$n.json)"
done
bash tools/tl_shard.sh gpurun_out/fin/tl8 8 || exit 1
bash tools/tl_shard.sh gpurun_out/fin/tl1 1 || exit 1
