"""Summarise a tools/profile.sh output directory into committed profile files.

    python tools/pmc_summary.py gpurun_out/prof profiles/r01

writes <prefix>_kernel_stats.csv (the rocprofv3 --stats table, unchanged),
<prefix>_pmc.csv (per-kernel mean of every collected counter) and
<prefix>_summary.json: per kernel the average duration (from --kernel-trace --stats)
and the HBM-side traffic per launch, corrected as MI355X_MICROARCH.md § HBM
prescribes: FETCH_SIZE (KiB) is doubled on gfx950, WRITE_SIZE (KiB) taken as is,
each from its own --pmc pass.
"""
from __future__ import annotations

import json
import os
import re
import shutil
import sys

import pandas as pd


F64_COUNTERS = ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64")


def short_name(name: str) -> str:
    """'void scde::k_boot2<20>(double const*, ...)' -> 'k_boot2<20>';
    'scde::(anonymous namespace)::k_prior_bin(int const*, ...)' -> 'k_prior_bin'."""
    n = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    return n.replace("scde::", "")


def load_counters(root: str) -> pd.DataFrame:
    frames = []
    for sub in sorted(os.listdir(root)):
        p = os.path.join(root, sub, "run_counter_collection.csv")
        if sub.startswith("pmc") and os.path.exists(p):
            d = pd.read_csv(p)
            d["pass"] = sub
            frames.append(d)
    if not frames:
        return pd.DataFrame()
    d = pd.concat(frames)
    d["kernel"] = d["Kernel_Name"].map(short_name)
    return d


def main(src: str, prefix: str) -> None:
    os.makedirs(os.path.dirname(prefix) or ".", exist_ok=True)
    stats_p = os.path.join(src, "trace", "run_kernel_stats.csv")
    stats = pd.read_csv(stats_p)
    shutil.copyfile(stats_p, prefix + "_kernel_stats.csv")
    stats["kernel"] = stats["Name"].map(short_name)
    cnt = load_counters(src)
    summary = {"source": src, "kernels": {}}
    pm = None
    if len(cnt):
        pm = cnt.groupby(["kernel", "Counter_Name"])["Counter_Value"].mean().unstack()
        pm.to_csv(prefix + "_pmc.csv")
    for _, r in stats.iterrows():
        k = r["kernel"]
        e = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6, "pct": float(r["Percentage"])}
        if pm is not None and k in pm.index:
            row = pm.loc[k]
            fetch = row.get("FETCH_SIZE")
            write = row.get("WRITE_SIZE")
            if pd.notna(fetch):
                e["fetch_bytes"] = float(fetch) * 1024 * 2  # KiB, x2 gfx950 correction
            if pd.notna(write):
                e["write_bytes"] = float(write) * 1024
            if pd.notna(fetch) and pd.notna(write):
                e["traffic_bytes"] = e["fetch_bytes"] + e["write_bytes"]
            hit, miss = row.get("TCC_HIT_sum"), row.get("TCC_MISS_sum")
            if pd.notna(hit) and pd.notna(miss) and hit + miss > 0:
                e["l2_hit"] = float(hit / (hit + miss))
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES", "SQ_INSTS_VALU",
                      "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD") + F64_COUNTERS:
                if c in row.index and pd.notna(row[c]):
                    e[c] = float(row[c])
            # FP64 VALU flops per launch from the gfx950 per-class instruction counters (wave
            # instructions x 64 lanes; an FMA counts 2), omniperf's formula
            if all(c in e for c in F64_COUNTERS):
                e["fp64_flops"] = 64.0 * (2.0 * e["SQ_INSTS_VALU_FMA_F64"] + e["SQ_INSTS_VALU_ADD_F64"] +
                                          e["SQ_INSTS_VALU_MUL_F64"] + e["SQ_INSTS_VALU_TRANS_F64"])
        summary["kernels"][k] = e
    with open(prefix + "_summary.json", "w") as f:
        json.dump(summary, f, indent=1, sort_keys=True)
    top = sorted(summary["kernels"].items(), key=lambda kv: -kv[1]["pct"])[:6]
    for k, e in top:
        print(f"{k:40s} {e['avg_ms']:8.3f} ms x{e['calls']:3d}  {e['pct']:5.1f}%  "
              f"traffic {e.get('traffic_bytes', float('nan')) / 1e9:7.3f} GB")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
