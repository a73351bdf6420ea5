#!/usr/bin/env python3
"""Per-dispatch PMC counters joined with kernel-trace durations, for the LONGEST dispatches whose
kernel name matches a substring.  usage: pmc_dispatch.py <substring> <top> <dir> [<dir> ...]
(each dir = one rocprofv3 --kernel-trace --pmc run over the same workload; dispatches are matched
by their order among the matching kernels, so every run must launch the same sequence)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d, pat, marker="sgd_kernel"):
    """Only dispatches of the LAST step (after the second-to-last `marker` kernel): warm-up steps
    include the autotuner's trial launches."""
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    dur = {}
    marks = []
    for f in kt:
        for r in csv.DictReader(open(f)):
            if marker in r.get("Kernel_Name", ""):
                marks.append(int(r["Dispatch_Id"]))
            if pat in r.get("Kernel_Name", ""):
                dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    marks.sort()
    lo = marks[-2] if len(marks) >= 2 else -1
    dur = {k: v for k, v in dur.items() if int(k) > lo}
    ctr = defaultdict(dict)
    names = {}
    for f in cc:
        for r in csv.DictReader(open(f)):
            if pat not in r.get("Kernel_Name", ""):
                continue
            did = r.get("Dispatch_Id") or r.get("Correlation_Id")
            if did not in dur:
                continue
            ctr[did][r["Counter_Name"]] = ctr[did].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            names[did] = (r["Kernel_Name"], r.get("Grid_Size", "?"))
    order = sorted(ctr, key=lambda x: int(x))
    return [(did, names[did], dur.get(did), ctr[did]) for did in order]


def main():
    pat, top, dirs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    runs = [load(d, pat) for d in dirs]
    n = min(len(r) for r in runs)
    rows = []
    for i in range(n):
        merged = {}
        for r in runs:
            merged.update(r[i][3])
        durs = [r[i][2] for r in runs if r[i][2] is not None]
        rows.append((sum(durs) / len(durs) if durs else 0.0, runs[0][i][1], merged))
    rows.sort(key=lambda x: -x[0])
    for us, (name, grid), c in rows[:top]:
        print(f"{us:9.1f} us  grid {grid}  {name[:110]}")
        for k in sorted(c):
            print(f"      {k:28s} {c[k]:16.0f}")
        # FETCH_SIZE / WRITE_SIZE are kilobytes
        if "FETCH_SIZE" in c and us:
            print(f"      HBM read  {c['FETCH_SIZE'] / 1e3:8.1f} MB  ({c['FETCH_SIZE'] * 1e-3 / us:5.2f} TB/s)")
        if "WRITE_SIZE" in c and us:
            print(f"      HBM write {c['WRITE_SIZE'] / 1e3:8.1f} MB  ({c['WRITE_SIZE'] * 1e-3 / us:5.2f} TB/s)")


if __name__ == "__main__":
    main()
