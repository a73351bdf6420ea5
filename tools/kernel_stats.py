#!/usr/bin/env python3
"""Per-kernel time summary from a rocprofv3 kernel trace (``--kernel-trace`` CSV or the rocpd
SQLite ``*_results.db``): total / per-step time per kernel family, share of GPU time, and the
share spent in mipipe's own HIP kernels vs anything else (ATen, rocclr copies / fills, RCCL).

usage: python tools/kernel_stats.py <trace.csv | results.db> [--steps N] [--top 25]
       (--steps: the number of steps the trace covers, to print per-step times; the warm-up
        steps in the trace can be excluded with --skip-until <kernel substring> --skip N)
"""
from __future__ import annotations

import argparse
import collections
import csv
import re
import sqlite3
import sys


def load(path):
    """-> list of (name, start_ns, end_ns) in start order."""
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        rows = [(n, s, e) for n, s, e in c.execute("select name, start, end from kernels")]
    else:
        rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: r[1])
    return rows


def family(name: str) -> str:
    """Collapse template arguments / signatures into a readable kernel family."""
    n = name
    if n.startswith("_Z"):
        m = re.match(r"_ZN6mipipe(?:2gk)?\d+([a-z_0-9]+?)I", n) or re.match(
            r"_ZN6mipipe(?:2gk)?\d+([a-z_0-9]+)", n)
        if m:
            n = "mipipe::" + m.group(1) + "<" + ("f32" if "EfE" in name or "fEE" in name else
                                                  "bf16") + ">"
    n = re.sub(r"\(.*$", "", n)
    n = n.replace("void ", "")
    if len(n) > 90:
        n = n[:90]
    return n


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=0)
    ap.add_argument("--step-marker", default="sgd_kernel",
                    help="kernel ending each step; with --last N only the last N steps count")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = load(a.trace)
    steps = a.steps
    if a.last:
        ends = [e for n, s, e in rows if a.step_marker in n]
        if len(ends) > a.last:
            t0 = ends[-a.last - 1]
            rows = [r for r in rows if r[1] >= t0]
        steps = a.last
    tot = collections.Counter()
    cnt = collections.Counter()
    for n, s, e in rows:
        f = family(n)
        tot[f] += e - s
        cnt[f] += 1
    all_ns = sum(tot.values())
    mip = sum(v for k, v in tot.items() if k.startswith("mipipe"))
    per = f" per step over {steps} steps" if steps else ""
    print(f"trace: {a.trace}")
    print(f"kernel time{per}: {all_ns / 1e6 / max(steps, 1):.3f} ms; mipipe HIP kernels "
          f"{mip / max(all_ns, 1) * 100:.1f} %, other {100 - mip / max(all_ns, 1) * 100:.1f} %")
    print(f"{'ms/step' if steps else 'ms':>9} {'share':>6} {'calls':>6}  kernel")
    for k, v in tot.most_common(a.top):
        print(f"{v / 1e6 / max(steps, 1):9.3f} {v / all_ns * 100:5.1f}% "
              f"{cnt[k] // max(steps, 1):6d}  {k}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
