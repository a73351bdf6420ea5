#!/usr/bin/env python3
"""Mean per-dispatch PMC counter values for kernels matching a substring, from rocprofv3
--pmc CSV output directories.  usage: pmc_summary.py <substring> <dir> [<dir> ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    pat, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(list)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            for r in csv.DictReader(open(f)):
                if pat not in r.get("Kernel_Name", ""):
                    continue
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
            for (disp, name), v in per.items():
                vals[name].append(v)
    for name in sorted(vals):
        v = vals[name]
        print(f"{name:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
    g = {k: sum(v) / len(v) for k, v in vals.items()}
    if "SQ_LDS_BANK_CONFLICT" in g and "SQ_LDS_IDX_ACTIVE" in g and g["SQ_LDS_IDX_ACTIVE"]:
        print(f"LDS bank-conflict share of LDS active cycles: {100 * g['SQ_LDS_BANK_CONFLICT'] / g['SQ_LDS_IDX_ACTIVE']:.1f}%")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in g and "SQ_BUSY_CYCLES" in g and g["SQ_BUSY_CYCLES"]:
        print(f"MFMA busy / SQ busy: {g['SQ_VALU_MFMA_BUSY_CYCLES'] / g['SQ_BUSY_CYCLES']:.2f}")


if __name__ == "__main__":
    main()
