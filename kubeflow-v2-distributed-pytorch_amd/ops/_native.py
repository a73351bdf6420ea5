"""Loader for the in-tree gfx950 extension ``mipipe/_C*.so`` (built by ``setup.py`` /
``__graft_entry__.build``).  The .so lives inside the package so the GPU box sees it."""
from __future__ import annotations

import glob
import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err = None


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        pkg_dir = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        if not glob.glob(os.path.join(pkg_dir, "_C*.so")):
            _err = FileNotFoundError(f"no _C*.so in {pkg_dir}")
            return
        try:
            import torch  # noqa: F401 - the extension links against libtorch
            _mod = importlib.import_module("mipipe._C")
        except Exception as e:  # pragma: no cover - depends on build
            _err = e


def native_available() -> bool:
    _load()
    return _mod is not None


def native():
    _load()
    if _mod is None:
        raise RuntimeError(f"mipipe._C not available: {_err!r}")
    return _mod


def load_error():
    _load()
    return _err
