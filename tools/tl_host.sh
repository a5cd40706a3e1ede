# host-path step timelines (GPU box): config 3 at N = 1 and rank 0's shard of 8
bash tools/tl_shard.sh gpurun_out/tlh1 1 --trace-host || exit 1
bash tools/tl_shard.sh gpurun_out/tlh8 8 --trace-host || exit 1
