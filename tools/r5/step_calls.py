"""Per-call kernel table of ONE training step from a rocprofv3 kernel trace.

usage: python tools/r5/step_calls.py <run_kernel_trace.csv | run_results.db> [--delim sgd_kernel] [--family]

The step is the span between the last two launches of the delimiter kernel (the optimizer).
Names are demangled with llvm-cxxfilt and shortened to kernel + tile; --family prints per-family
totals instead of the call list.
"""
import argparse
import csv
import re
import subprocess
from collections import defaultdict

CXXFILT = "c++filt"


def demangle(names):
    p = subprocess.run([CXXFILT], input="\n".join(n.replace("DF16b", "u4bf16") for n in names), capture_output=True, text=True)
    return p.stdout.splitlines()


def short(n):
    n = n.replace("mipipe::", "").replace("gk::", "").replace("__hip_bfloat16", "bf16")
    m = re.match(r"(?:void )?([\w:]+)", n)
    base = m.group(1) if m else n[:40]
    t = re.findall(r"Tile<([\d, ]+), (true|false)>", n)
    if t:
        base += "[" + t[0][0].replace(" ", "") + ("pp" if t[0][1] == "true" else "") + "]"
    return base


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--delim", default="sgd_kernel")
    ap.add_argument("--family", action="store_true")
    a = ap.parse_args()
    if a.trace.endswith(".db"):  # rocprofv3's default SQLite output
        import sqlite3
        cur = sqlite3.connect(a.trace).execute(
            "select name, start, end, grid_x, workgroup_x, grid_y, vgpr_count, accum_vgpr_count, "
            "lds_size from kernels")
        keys = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Workgroup_Size_X",
                "Grid_Size_Y", "VGPR_Count", "Accum_VGPR_Count", "LDS_Block_Size"]
        rows = [dict(zip(keys, map(str, r))) for r in cur]
    else:
        rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = demangle([r["Kernel_Name"] for r in rows])
    idx = [i for i, n in enumerate(names) if a.delim in n]
    lo, hi = idx[-2] + 1, idx[-1] + 1
    fam = defaultdict(lambda: [0.0, 0])
    tot = 0.0
    for r, n in zip(rows[lo:hi], names[lo:hi]):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot += d
        s = short(n)
        fam[s][0] += d
        fam[s][1] += 1
        if not a.family:
            g = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
            print(f"{d:8.1f} {s[:44]:44s} grid={g}x{r['Grid_Size_Y']} wg={r['Workgroup_Size_X']} "
                  f"vgpr={r['VGPR_Count']}/{r['Accum_VGPR_Count']} lds={r['LDS_Block_Size']}")
    if a.family:
        for k, (t, c) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
            print(f"{t:9.1f} us {100 * t / tot:5.1f}% {c:4d}  {k}")
    print(f"step kernel time {tot:.1f} us ({hi - lo} launches)")


if __name__ == "__main__":
    main()
