#!/bin/bash
# final build: GPU suite, smoke(), then the default bench line
set -o pipefail
bash tools/r5_check.sh || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r5check/bench.json 2> gpurun_out/r5check/bench.err || { tail -5 gpurun_out/r5check/bench.err; exit 1; }
grep -o '"value": [0-9.e+]*\|"ms_per_step": [0-9.e+]*\|"frac": [0-9.e+]*' gpurun_out/r5check/bench.json | tr '\n' ' '
