"""Timeline of one bench step from a rocprofv3 kernel + memory-copy trace (GPU box):

  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d OUT -o run -- python3 bench.py ...
  python tools/timeline.py OUT [steps]

prints the last step's kernels and copies in start order with the idle gaps between them
(a step = the span from the first k_cell_prep launch of a call to the next one)."""
import csv
import glob
import sys


def load(out):
    rows = []
    for kind, pat in (("K", "*kernel_trace.csv"), ("C", "*memory_copy_trace.csv")):
        for f in glob.glob(out + "/**/" + pat, recursive=True):
            for r in csv.DictReader(open(f)):
                name = r.get("Kernel_Name") or (r.get("Direction", "copy") + " " + r.get("Size", ""))
                name = name.split("(")[0].replace("void ", "").replace("scde::", "")
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name))
    # host API calls (a --hip-runtime-trace run): the syncs and copies, with the issuing thread
    keep = ("Synchronize", "Memcpy", "EventQuery", "HostMalloc", "Malloc", "Free")
    for f in glob.glob(out + "/**/*hip_api_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            fn = r.get("Function", "")
            if any(k in fn for k in keep):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "A",
                             f"{fn} [thread {r.get('Thread_Id', '?')}]"))
    rows.sort()
    return rows


def main():
    out = sys.argv[1]
    rows = load(out)
    starts = [i for i, r in enumerate(rows) if r[2] == "K" and "k_cell_prep" in r[3]]
    # (with API rows, a step starts at the first API call after the previous step's last kernel)
    # two k_cell_prep per DE call (one per group): a step starts at every other one
    steps = starts[::2]
    a, b = steps[-2], steps[-1]
    seg = rows[a:b]
    t0 = seg[0][0]
    busy_end = t0
    idle = 0
    for s, e, k, n in seg:
        if k == "A":  # host API call: printed, not part of the device's busy time
            print(f"{(s - t0) / 1e3:9.1f} us  {'':13s}  {(e - s) / 1e3:8.1f} us  {k} {n[:70]}")
            continue
        gap = max(0, s - busy_end)
        idle += gap
        busy_end = max(busy_end, e)
        print(f"{(s - t0) / 1e3:9.1f} us  +{gap / 1e3:7.1f} gap  {(e - s) / 1e3:8.1f} us  {k} {n[:70]}")
    span = rows[b][0] - t0
    print(f"span {span / 1e3:.1f} us, idle {idle / 1e3:.1f} us")


if __name__ == "__main__":
    main()
