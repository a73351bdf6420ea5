#!/usr/bin/env python3
"""Per-call listing of ONE training step from a rocprofv3 kernel trace (CSV): every kernel in
launch order with its duration, grid and tile config, plus the gap to the previous kernel.

usage: python tools/r2/per_call.py <run_kernel_trace.csv> [--marker sgd_kernel] [--min-us 0]
The step is the span between the last two `--marker` kernels (the optimizer ends each step).
"""
from __future__ import annotations

import argparse
import csv
import re
import sys


def short(name: str) -> str:
    n = re.sub(r"\(.*$", "", name).replace("void ", "").replace("mipipe::", "").replace("gk::", "")
    n = n.replace("__bf16", "bf16")
    m = re.match(r"(\w+)<Tile<(\d+), (\d+), (\d+), (\d+), (\d+)>, (.*)>$", n)
    if m:
        k, bm, bn, ns, wm, wn, rest = m.groups()
        return f"{k} {bm}x{bn}/s{ns}/{wm}x{wn} <{rest}>"
    return n[:110]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="sgd_kernel")
    ap.add_argument("--min-us", type=float, default=0.0)
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        def dim(prefix):  # total over x, y, z (split-K weight-grads launch (tiles, splits, 1))
            if prefix + "_X" in r:
                v = 1
                for ax in "XYZ":
                    v *= max(1, int(r.get(f"{prefix}_{ax}", 1) or 1))
                return v
            return int(r.get(prefix, 0) or 0)
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     dim("Grid_Size"), dim("Workgroup_Size"),
                     r.get("VGPR_Count", r.get("Arch_VGPR_Count", "")),
                     r.get("LDS_Block_Size", r.get("LDS_Size", ""))))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(ends) < 2:
        print("fewer than two step markers in the trace", file=sys.stderr)
        return 1
    step = rows[ends[-2] + 1: ends[-1] + 1]
    tot = sum(e - s for s, e, *_ in step)
    span = step[-1][1] - step[0][0]
    print(f"step: {len(step)} kernels, kernel time {tot / 1e3:.1f} us, span {span / 1e3:.1f} us")
    print(f"{'#':>4} {'us':>8} {'gap':>6} {'wgs':>7} {'thr':>4} {'vgpr':>5} {'lds':>6}  kernel")
    prev_end = step[0][0]
    for i, (s, e, n, grid, wg, vg, lds) in enumerate(step):
        us = (e - s) / 1e3
        gap = (s - prev_end) / 1e3
        prev_end = e
        if us < a.min_us:
            continue
        wgs = grid // wg if wg else grid  # workgroups of the whole grid (x*y*z)
        print(f"{i:4d} {us:8.1f} {gap:6.1f} {wgs:7d} {wg:4d} {vg:>5} {lds:>6}  {short(n)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
