#!/usr/bin/env python3
"""Collective / compute overlap report from a rocprofv3 ``--kernel-trace`` CSV.

For every RCCL kernel (all-reduce / one-rank reduce / broadcast ...) it reports when it ran
relative to the backward's conv dgrad / wgrad kernels and how much of its duration overlapped
compute kernels on other streams.  Evidence for SURVEY C5 (bucketed all-reduce overlapped with
backward): buckets must launch *between* backward GEMMs, not after the last one.

usage: python tools/overlap_report.py <kernel_trace.csv> [--steps N]
"""
from __future__ import annotations

import argparse
import csv
import sys


def is_comm(name: str) -> bool:
    n = name.lower()
    return "nccl" in n or "rccl" in n or "onerankreduce" in n or "allreduce" in n


def is_bwd_gemm(name: str) -> bool:
    return "conv_dgrad" in name or "conv_wgrad" in name or "gemm_dense" in name


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step-marker", default="sgd_kernel",
                    help="kernel that ends a training step (optimizer)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    for r in rows:
        r["t0"] = int(r["Start_Timestamp"])
        r["t1"] = int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["t0"])
    ends = [r["t1"] for r in rows if a.step_marker in r["Kernel_Name"]]
    if len(ends) < 2:
        print("fewer than 2 steps in trace", file=sys.stderr)
        return 1
    print(f"trace: {a.csv}")
    print(f"steps: {len(ends)} (delimited by '{a.step_marker}')")
    tot_comm = tot_ovl = 0.0
    for s in range(1, len(ends)):
        lo, hi = ends[s - 1], ends[s]
        step = [r for r in rows if lo <= r["t0"] < hi]
        comm = [r for r in step if is_comm(r["Kernel_Name"])]
        comp = [r for r in step if not is_comm(r["Kernel_Name"])]
        bwd = [r for r in step if is_bwd_gemm(r["Kernel_Name"])]
        if not bwd:
            continue
        first_bwd, last_bwd = min(r["t0"] for r in bwd), max(r["t1"] for r in bwd)
        lines = []
        for c in comm:
            ovl = 0
            for k in comp:
                if k["Stream_Id"] == c["Stream_Id"]:
                    continue
                ovl += max(0, min(c["t1"], k["t1"]) - max(c["t0"], k["t0"]))
            dur = c["t1"] - c["t0"]
            n_after = sum(1 for r in bwd if r["t0"] > c["t1"])
            tot_comm += dur
            tot_ovl += min(ovl, dur)
            lines.append(f"    +{(c['t0'] - lo) / 1e3:8.1f} us  dur {dur / 1e3:7.1f} us  "
                         f"overlapped {min(ovl, dur) / max(dur, 1) * 100:5.1f}%  "
                         f"backward GEMMs still to run after it: {n_after:3d}  "
                         f"stream {c['Stream_Id']}  {c['Kernel_Name'][:60]}")
        print(f"  step {s}: {(hi - lo) / 1e3:.1f} us, backward GEMMs {len(bwd)} "
              f"[{(first_bwd - lo) / 1e3:.1f} .. {(last_bwd - lo) / 1e3:.1f}] us, "
              f"collectives {len(comm)}")
        print("\n".join(lines))
    if tot_comm:
        print(f"collective time overlapped with compute on other streams: "
              f"{tot_ovl / tot_comm * 100:.1f}% of {tot_comm / 1e3:.1f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())
