"""roctx ranges around training-step phases (data, fwd, bwd, allreduce-wait,
optimizer) so ``rocprofv3 --marker-trace --kernel-trace`` attributes every HIP kernel to a
phase.  Enabled by ``MIPIPE_TRACE=1`` (or :func:`enable`); otherwise ``phase()`` is a no-op
context manager costing one attribute check.

The ranges go straight to ROCm's ``libroctx64`` through ctypes (no torch profiler involved),
mirrored into ``torch.profiler.record_function`` when a torch profiler is active.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
from typing import Optional

_lib: Optional[ctypes.CDLL] = None
_enabled = os.environ.get("MIPIPE_TRACE", "0") == "1"


def _load() -> Optional[ctypes.CDLL]:
    global _lib
    if _lib is None:
        for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _lib = lib
                break
            except OSError:
                continue
    return _lib


def enable(on: bool = True) -> bool:
    """Turn phase ranges on/off; returns whether roctx is available."""
    global _enabled
    _enabled = on
    return _load() is not None


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def phase(name: str):
    if not _enabled:
        yield
        return
    lib = _load()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        import torch
        with torch.profiler.record_function(name):
            yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(msg: str) -> None:
    if _enabled:
        lib = _load()
        if lib is not None:
            lib.roctxMarkA(msg.encode())
