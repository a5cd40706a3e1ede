# final bench lines of the session (GPU box): GPU suite + smoke, then configs 3, 4, 2b and the config-3 shards
bash tools/final_check.sh || exit 1
for c in 3 4 2b; do
  timeout -k 10 400 python bench.py --config $c > gpurun_out/fin/b_$c.json 2> gpurun_out/fin/b_$c.err || { tail -5 gpurun_out/fin/b_$c.err; exit 1; }
  echo "config $c: $(grep -o '"ms_per_step": [0-9.e+]*\|device_resident_ms_per_step": [0-9.e+]*' gpurun_out/fin/b_$c.json | tr '\n' ' ')"
done
