#!/bin/bash
# Shard-of-N bench lines of config 3 (rank 0's shard of an N-way split, one process) and the
# N = 1 / N = 8 step timelines: tools/measure_shards.sh TAG
TAG=$1
mkdir -p gpurun_out/fin
for n in 2 4 8; do
  timeout -k 10 300 python bench.py --config 3 --shard-of $n --cpu-sample 0 > gpurun_out/fin/b_3_shard_of_$n.json 2> gpurun_out/fin/b_3_shard_$n.err || { tail -5 gpurun_out/fin/b_3_shard_$n.err; exit 1; }
  echo "shard of $n: $(grep -o '"ms_per_step": [0-9.e+]*' gpurun_out/fin/b_3_shard_of_$n.json) $(grep -o '"device_resident_ms_per_step": [0-9.e+]*' gpurun_out/fin/b_3_shard_of_$n.json)"
done
bash tools/tl_api.sh gpurun_out/fin/tl1 1 || exit 1
bash tools/tl_api.sh gpurun_out/fin/tl8 8 || exit 1
echo shards done
