"""Per-shape kernel selection: mipipe's analogue of ``torch.backends.cudnn.benchmark``.

The reference turns cuDNN's autotuner on (``cudnn.benchmark = True``, /root/reference/task.py:244)
so every convolution shape runs its fastest algorithm.  mipipe's convolutions are implicit GEMMs
over a table of tile configs (block tile, LDS stages, 4- or 8-wave grid —
csrc/kernels/conv_common.hpp).  With benchmark mode on, the first eager call of a conv op on a new
(op, shape, dtype) times every valid config on scratch outputs and caches the fastest; calls made
while a stream is being captured into a hipGraph never tune (they use the cache or the
heuristic), so tuning happens in the warm-up steps before capture.

The table is plain data (``{"fwd|N,H,W,Ci,Co,KH,KW,s,p,sw,pw|bf16": cfg}``): :func:`save` /
:func:`load` persist it so a job can start from a measured table (no re-tuning per rank).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional

from ._native import native, native_available

__all__ = ["set_benchmark", "benchmark_enabled", "table", "load", "save", "clear"]


def set_benchmark(on: bool = True, verbose: bool = False, reps: int = 3) -> None:
    """Enable / disable per-shape tile autotuning (no-op without the native extension)."""
    if native_available():
        native().set_benchmark(bool(on), bool(verbose), int(reps))


def benchmark_enabled() -> bool:
    return native_available() and bool(native().get_benchmark())


def table() -> Dict[str, int]:
    return dict(native().tune_table()) if native_available() else {}


def load(src) -> int:
    """Merge entries from a dict or a JSON file path; returns the number of entries loaded."""
    if not native_available():
        return 0
    if isinstance(src, (str, os.PathLike)):
        with open(src) as f:
            src = json.load(f)
    n = 0
    for k, v in src.items():
        native().set_tune_entry(str(k), int(v))
        n += 1
    return n


def save(path: str) -> None:
    with open(path, "w") as f:
        json.dump(table(), f, indent=1, sort_keys=True)


def clear() -> None:
    if native_available():
        native().clear_tune_table()


def from_env() -> Optional[str]:
    """``MIPIPE_TUNE_TABLE=path``: load a saved table at import of the training entry points."""
    p = os.environ.get("MIPIPE_TUNE_TABLE")
    if p and os.path.exists(p):
        load(p)
        return p
    return None
