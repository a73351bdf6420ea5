"""Per-kernel load / full-drain audit of a HIP source compiled for gfx950.

A global load behind a runtime branch is closed by hipcc with ``s_waitcnt vmcnt(0)``: every
load in flight is waited for right there (profiles/r3_experiments.md).  This lists, per kernel,
the global/buffer loads, the full vmcnt(0) drains, VGPRs and scratch spills of the device
assembly, so kernels that drain after nearly every load stand out.

usage: python tools/r3/drain_audit.py csrc/kernels/bn.hip [--filter bn_] [--min-ratio 0.0]
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile


def audit(src: str, flt: str):
    inc = os.path.dirname(os.path.abspath(src))
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-S",
                        "--cuda-device-only", "-I" + inc, src, "-o", out], check=True,
                       stderr=subprocess.DEVNULL)
        text = open(out).read()
    stats, cur = {}, None
    for line in text.split("\n"):
        m = re.match(r"^(_Z\w+):", line)
        if m:
            cur = m.group(1)
            stats[cur] = [0, 0, 0, 0]
            continue
        if cur and line.startswith(".Lfunc_end"):
            cur = None
            continue
        if cur:
            if "s_waitcnt vmcnt(0)" in line:
                stats[cur][1] += 1
            if re.search(r"\b(global|buffer)_load", line):
                stats[cur][0] += 1
    for m in re.finditer(r"\.name:\s+(_Z\w+)\n((?:.*\n){0,60}?)\s+\.vgpr_count:\s+(\d+)\n(?:.*\n){0,5}?\s+\.vgpr_spill_count:\s+(\d+)", text):
        if m.group(1) in stats:
            stats[m.group(1)][2:] = [int(m.group(3)), int(m.group(4))]
    return {k: v for k, v in stats.items() if flt in k}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    ap.add_argument("--min-ratio", type=float, default=0.0)
    a = ap.parse_args()
    rows = audit(a.src, a.filter)
    print(f"{'loads':>6} {'drains':>6} {'vgpr':>5} {'spill':>5}  kernel")
    for k, (ld, dr, vg, sp) in sorted(rows.items(), key=lambda kv: -kv[1][1]):
        if ld and dr / ld < a.min_ratio:
            continue
        print(f"{ld:6d} {dr:6d} {vg:5d} {sp:5d}  {k[:110]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
