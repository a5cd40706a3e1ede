export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/p4 -o run -- python3 tools/qdiag.py 4 > gpurun_out/p4.log 2>&1
