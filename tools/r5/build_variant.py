#!/usr/bin/env python3
"""Build an A/B variant of mipipe/_C with extra compile definitions into tools/r5/alt/<name>/
(a full package copy is assembled on the GPU box by tools/r5/ab_run.sh).

python tools/r5/build_variant.py NAME -DFLAG [-DFLAG ...]"""
import glob
import os
import sys
import concurrent.futures as cf

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from tools import build_ext as B  # noqa: E402


def main():
    name, defs = sys.argv[1], sys.argv[2:]
    out_dir = os.path.join(B.REPO, "tools", "r5", "alt", name)
    obj_dir = os.path.join(B.REPO, "build", "obj_" + name)
    os.makedirs(out_dir, exist_ok=True)
    os.makedirs(obj_dir, exist_ok=True)
    tflags, ldflags = B._torch_flags()
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{B.CSRC}", "-DNDEBUG", "-Wno-unused-result"] + defs
    hip_flags = common + [f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics"] + tflags
    jobs = []
    for s in sorted(glob.glob(os.path.join(B.CSRC, "kernels", "*.hip"))):
        jobs.append((s, os.path.join(obj_dir, os.path.basename(s) + ".o"), hip_flags))
    for s in [os.path.join(B.CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(B.CSRC, "comm", "*.cpp"))):
        jobs.append((s, os.path.join(obj_dir, os.path.basename(s) + ".o"), common + tflags))
    with cf.ThreadPoolExecutor(8) as ex:
        list(ex.map(lambda j: B._run([B.HIPCC] + j[2] + ["-c", j[0], "-o", j[1]]), jobs))
    out = os.path.join(out_dir, "_C" + B.EXT)
    B._run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}"] + [j[1] for j in jobs] +
           ldflags + ["-o", out])
    print(out)


if __name__ == "__main__":
    main()
