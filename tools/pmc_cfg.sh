#!/bin/bash
# One PMC pass (8 SQ counters) over a short bench run: tools/pmc_cfg.sh OUTDIR "COUNTERS" BENCH_ARGS...
out=$1; ctr=$2; shift 2
export TMPDIR=/tmp
mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $out/pmc -o run -- python3 bench.py "$@" > $out/pmc.log 2>&1 || exit 1
python3 - $out <<'PY'
import csv, glob, sys, collections
rows = []
for f in glob.glob(sys.argv[1] + "/pmc/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in sorted(agg.items(), key=lambda x: -x[1].get("SQ_WAVE_CYCLES", 0))[:10]:
    n = max(cnt[(k, c)] for c in d)
    print(k, {c: f"{v / n:.4g}" for c, v in d.items()}, "launches", n)
PY
