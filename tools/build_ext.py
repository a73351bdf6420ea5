"""Build mipipe's native code for gfx950 with hipcc directly (no hipify, no JIT cache).

Products (in-tree, so they travel to the GPU box with the repo snapshot):
  mipipe/_C<EXT_SUFFIX>      torch extension: HIP kernels (csrc/kernels/*.hip) + bindings
  mipipe/_runtime<EXT_SUFFIX> native runtime (csrc/runtime/*.cpp): process supervisor,
                              DAG scheduler core (CPython API, no torch)

Incremental: an object is rebuilt when its source or any header under csrc/ is newer.  On top of
the mtimes, each linked library records the SHA-256 of the sources it was built from
(``<lib>.srcsha``, next to it): a library whose sources changed — or that arrived without a
stamp, e.g. a snapshot with stale mtimes — is rebuilt from scratch, and ``MIPIPE_FORCE_BUILD=1``
(or ``--force``) always rebuilds everything.  Every build appends one line to
``build/provenance.jsonl`` (library, digest, objects compiled / reused, forced or not).
Usage: python tools/build_ext.py [-j N] [--force] [--only C|runtime]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import subprocess
import sys
import sysconfig

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "csrc")
PKG = os.path.join(REPO, "kubeflow-v2-distributed-pytorch_amd")
BUILD = os.path.join(REPO, "build", "obj")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _newest_header() -> float:
    hs = glob.glob(os.path.join(CSRC, "**", "*.hpp"), recursive=True) + \
        glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)
    return max([os.path.getmtime(h) for h in hs] or [0.0])


def sources_digest(kind: str) -> str:
    """SHA-256 over the sources (paths + bytes) a library is built from."""
    if kind == "C":
        pats = ["kernels/*.hip", "kernels/*.hpp", "bindings.cpp", "comm/*.cpp", "comm/*.h*"]
    else:
        pats = ["runtime/*.cpp", "runtime/*.h*"]
    files = sorted({f for p in pats for f in glob.glob(os.path.join(CSRC, p))})
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.relpath(f, CSRC).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(ARCH.encode())
    return h.hexdigest()


def _stamp_ok(lib: str, digest: str) -> bool:
    try:
        with open(lib + ".srcsha") as f:
            return os.path.exists(lib) and f.read().strip() == digest
    except OSError:
        return False


def _record(lib: str, digest: str, msgs, forced: bool) -> None:
    with open(lib + ".srcsha", "w") as f:
        f.write(digest + "\n")
    os.makedirs(os.path.dirname(BUILD), exist_ok=True)
    import time
    rec = {"time": time.strftime("%Y-%m-%dT%H:%M:%S"), "lib": os.path.relpath(lib, REPO),
           "sha256": digest, "arch": ARCH, "forced": forced,
           "compiled": sum(m.startswith("compiled") for m in msgs),
           "up_to_date": sum(m.startswith("up-to-date") for m in msgs)}
    with open(os.path.join(os.path.dirname(BUILD), "provenance.jsonl"), "a") as f:
        f.write(json.dumps(rec) + "\n")


def _torch_flags():
    import torch
    import torch.utils.cpp_extension as ce
    inc = ce.include_paths(device_type="cuda")
    flags = [f"-I{p}" for p in inc]
    flags += [f"-I{sysconfig.get_paths()['include']}"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    flags += [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H",
              "-DTORCH_EXTENSION_NAME=_C", "-DUSE_ROCM=1"]
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    ldflags = [f"-L{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip",
               "-ltorch_hip", f"-Wl,-rpath,{libdir}"]
    return flags, ldflags


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _compile(src: str, obj: str, flags, force: bool, hdr_time: float) -> str:
    if not force and os.path.exists(obj):
        t = os.path.getmtime(obj)
        if t >= os.path.getmtime(src) and t >= hdr_time:
            return f"up-to-date {os.path.relpath(src, REPO)}"
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    _run([HIPCC] + flags + ["-c", src, "-o", obj])
    return f"compiled {os.path.relpath(src, REPO)}"


def build_kernels(jobs: int = 8, force: bool = False, verbose: bool = True) -> str:
    out = os.path.join(PKG, "_C" + EXT)
    digest = sources_digest("C")
    force = force or os.environ.get("MIPIPE_FORCE_BUILD") == "1" or not _stamp_ok(out, digest)
    tflags, ldflags = _torch_flags()
    common = ["-O3", "-std=c++17", "-fPIC", f"-I{CSRC}", "-DNDEBUG", "-Wno-unused-result"]
    hip_flags = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics"] + tflags
    cpp_flags = common + tflags
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpps = [os.path.join(CSRC, "bindings.cpp")] + sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp")))
    hdr = _newest_header()
    jobs_list = []
    for s in srcs:
        jobs_list.append((s, os.path.join(BUILD, "C", os.path.basename(s) + ".o"), hip_flags))
    for s in cpps:
        jobs_list.append((s, os.path.join(BUILD, "C", os.path.basename(s) + ".o"), cpp_flags))
    msgs = []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, o, f, force, hdr) for (s, o, f) in jobs_list]
        for fu in futs:
            msg = fu.result()
            msgs.append(msg)
            if verbose:
                print(msg, flush=True)
    objs = [o for (_, o, _) in jobs_list]
    if force or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + ldflags + ["-o", out])
        if verbose:
            print(f"linked {os.path.relpath(out, REPO)}", flush=True)
    _record(out, digest, msgs, force)
    return out


def build_runtime(jobs: int = 8, force: bool = False, verbose: bool = True) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    if not srcs:
        return ""
    py_inc = sysconfig.get_paths()["include"]
    import pybind11
    flags = ["-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden", f"-I{py_inc}",
             f"-I{pybind11.get_include()}", f"-I{CSRC}", "-Wall", "-Wno-unused-result"]
    hdr = _newest_header()
    out = os.path.join(PKG, "_runtime" + EXT)
    digest = sources_digest("runtime")
    force = force or os.environ.get("MIPIPE_FORCE_BUILD") == "1" or not _stamp_ok(out, digest)
    objs, msgs = [], []
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = []
        for s in srcs:
            o = os.path.join(BUILD, "runtime", os.path.basename(s) + ".o")
            objs.append(o)
            futs.append(ex.submit(_compile_cxx, s, o, flags, force, hdr))
        for fu in futs:
            msg = fu.result()
            msgs.append(msg)
            if verbose:
                print(msg, flush=True)
    if force or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        _run(["g++", "-shared", "-fPIC"] + objs + ["-o", out, "-lpthread"])
        if verbose:
            print(f"linked {os.path.relpath(out, REPO)}", flush=True)
    _record(out, digest, msgs, force)
    return out


def _compile_cxx(src, obj, flags, force, hdr_time):
    if not force and os.path.exists(obj):
        t = os.path.getmtime(obj)
        if t >= os.path.getmtime(src) and t >= hdr_time:
            return f"up-to-date {os.path.relpath(src, REPO)}"
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    _run(["g++"] + flags + ["-c", src, "-o", obj])
    return f"compiled {os.path.relpath(src, REPO)}"


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["C", "runtime"], default=None)
    a = ap.parse_args(argv)
    if a.only in (None, "runtime"):
        build_runtime(a.jobs, a.force)
    if a.only in (None, "C"):
        build_kernels(a.jobs, a.force)
    return 0


if __name__ == "__main__":
    sys.exit(main())
