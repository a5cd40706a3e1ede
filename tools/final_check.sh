# end-of-session check (GPU box): full GPU suite, smoke(), config-3 shard projections
mkdir -p gpurun_out/fin
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/fin/gputests.log 2>&1 || { tail -20 gpurun_out/fin/gputests.log; exit 1; }
tail -1 gpurun_out/fin/gputests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
for n in 2 4 8; do
timeout -k 10 200 python bench.py --config 3 --shard-of $n --cpu-sample 0 --cpu-workers 0 > gpurun_out/fin/b_3_shard_of_$n.json 2> gpurun_out/fin/b_3_shard_$n.err || exit 1
echo "shard-of $n: $(grep -o '"ms_per_step": [0-9.e+]*\|device_resident_ms_per_step": [0-9.e+]*' gpurun_out/fin/b_3_shard_of_$n.json | tr '\n' ' ')"
done
