mkdir -p gpurun_out/r5b
for f in tests/test_gpu_configs.py tests/test_gpu_fullsize.py; do
  timeout -k 10 300 python -u -m pytest $f tests/test_gpu_skip.py -q --timeout 200 --timeout-method thread -k "not skip_modes" > gpurun_out/r5b/bis.log 2>&1
  echo "$f: $(tail -1 gpurun_out/r5b/bis.log)"
done
for k in "whole_table" "config4" "config2b" "call_history"; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_skip.py -q --timeout 200 --timeout-method thread -k "$k or layouts" > gpurun_out/r5b/bis.log 2>&1
  echo "$k: $(tail -1 gpurun_out/r5b/bis.log)"
done
