#!/bin/bash
# fused two-group posteriors + tile-row stretch bootstrap: GPU suite, then A/B bench lines on one box
set -o pipefail
mkdir -p gpurun_out/r5b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r5b/gputests.log 2>&1; rc=$?
tail -3 gpurun_out/r5b/gputests.log; [ $rc -eq 0 ] || exit $rc
run() {  # tag, bench args...
  local tag=$1; shift
  timeout -k 10 300 python bench.py "$@" --steps 20 --warmup 3 --cpu-sample 0 --cpu-workers 0 > gpurun_out/r5b/b_$tag.json 2> gpurun_out/r5b/b_$tag.err || { tail -5 gpurun_out/r5b/b_$tag.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/r5b/b_$tag.json'))
k=d['kernel_ms_per_step']; h=d['host_syncs']['host_phase_ms_per_step']
print('$tag', 'host %.3f dev %.3f' % (d['ms_per_step'], d['device_resident_ms_per_step']), 'kern', {a: round(b,3) for a,b in k.items()}, 'hostph', {a: round(b,3) for a,b in h.items()})"
}
run c3_f1 --config 3
run c3_f0 --config 3 --opt fuse_groups=0
run s8_f1 --config 3 --shard-of 8
run s8_f0 --config 3 --shard-of 8 --opt fuse_groups=0

run s8_p2 --config 3 --shard-of 8 --opt pipeline_mb=0 --opt pieces=1


run c2_f1_r1 --config 2
run c2_f1_r0 --config 2 --opt boot2_rows=0
run c2_f0_r0 --config 2 --opt fuse_groups=0 --opt boot2_rows=0
run c2b_r1 --config 2b
run c2b_r0 --config 2b --opt boot2_rows=0
echo main done
# k_boot_gene timing builds (results wrong by construction): 16 no bound pass, 32 no row loop, 64 rows only
for d in 16 32 64; do
  SCDE_LIB=diag/libt$d.so run c3_diag$d --config 3 --opt lanes=1
done
echo diag done
