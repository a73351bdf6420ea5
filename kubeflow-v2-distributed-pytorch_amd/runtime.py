"""Access to the native host runtime ``mipipe/_runtime*.so`` (csrc/runtime/*.cpp):

* :class:`ProcessGroup`  — posix_spawn-based rank supervisor with fail-fast teardown
  (used by :func:`mipipe.launch.launcher.launch`);
* :class:`DagScheduler`  — pipeline DAG state machine (used by the orchestrator);
* :class:`RecordLoader`  — multi-threaded, memory-mapped record loader with augmentation
  (used by :mod:`mipipe.data.records`).

The module is built by ``tools/build_ext.py`` / ``__graft_entry__.build`` with g++ (no GPU
needed).  ``MIPIPE_NO_NATIVE_RUNTIME=1`` forces the pure-Python fallbacks (used by tests to
check both paths agree).
"""
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
        pkg = os.path.dirname(os.path.abspath(__file__))
        if not glob.glob(os.path.join(pkg, "_runtime*.so")):
            _err = FileNotFoundError(f"no _runtime*.so in {pkg} (run tools/build_ext.py)")
            return
        try:
            _mod = importlib.import_module("mipipe._runtime")
        except Exception as e:  # pragma: no cover
            _err = e


def runtime_available() -> bool:
    if os.environ.get("MIPIPE_NO_NATIVE_RUNTIME") == "1":
        return False
    _load()
    return _mod is not None


def runtime():
    if not runtime_available():
        raise RuntimeError(f"mipipe._runtime not available: {_err!r}")
    return _mod
