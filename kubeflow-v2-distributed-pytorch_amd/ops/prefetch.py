"""GEMM operand prefetch into the memory-side cache.

A GEMM whose operands were last touched milliseconds earlier reads them from HBM instead of the
256 MB memory-side cache (MALL), and the narrow-grid GEMMs of a transformer layer are latency
bound enough to feel it: BERT-base's FFN-out forward (4096 x 768, K = 3072) runs 34 us with both
operands cache-resident, 44 us with a cold weight and 51 us with both cold
(``tools/r6/fc2_probe2.py``, ``profiles/r6_gemm_cold_operands.txt``).  Inside a training step the
activation operand was just written by the previous kernel (warm); the weight was last read one
pass earlier (cold).

So GEMM *i* warms the weight of GEMM *i + 1*: its blocks each issue one load per 64-B line of a
share of that weight before their own main loop (``EpiParams::pf_*`` in ``csrc/kernels/gemm.hip``;
nothing is written).  The data-grad GEMM of a Linear also warms the saved input its weight-grad
GEMM reads right after it.  The weight order is recorded over one step (weights are persistent
tensors: the flat space's bf16 shadows, safe to hold and to read at any time) and replayed from
the next; a step whose GEMM sequence differs (an evaluation pass, another shape) stops it until
a new recording.  Same-stream and in-kernel: no fork / join, so nothing changes for hipGraph
capture.  (A side-stream touch kernel was tried first: ROCm serialised the graph's branches and
BERT-base lost 17 %, ``profiles/r6_prefetch_side_stream_negative.txt``.)

Handing saved tensors forward as well (the GELU pre-activation, the attention's packed q/k/v, a
LayerNorm's input, each warmed by the weight-grad GEMM that runs right before its backward) made
those hosting GEMMs slower than the backward kernels gained: 4,720 vs 4,849 seq/s without it, same
box (``profiles/r6_prefetch_handover_negative.txt``).

``MIPIPE_PREFETCH=0`` disables it.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

__all__ = ["step_boundary", "before_weight_gemm", "reset", "enabled"]

_MODE = os.environ.get("MIPIPE_PREFETCH", "1")


class _State:
    def __init__(self):
        self.order: List[torch.Tensor] = []  # weight operand per weight-GEMM, in step order
        self.recording = False
        self.armed = False
        self.cursor = 0
        self.volatile: set = set()  # order slots whose operand is re-made every step


_S = _State()


def enabled() -> bool:
    return _MODE != "0"


def reset() -> None:
    """Forget the recorded order (model / batch shape changed)."""
    _S.order, _S.recording, _S.armed, _S.cursor = [], False, False, 0
    _S.volatile = set()


def step_boundary() -> None:
    """Start of a training step (called by the flat optimizer's zero_grad): finish a recording
    (or start one) and rewind the cursor."""
    if not _S.order and not _S.recording:
        _S.recording = True
        return
    if _S.recording:
        _S.recording = False
        _S.armed = len(_S.order) > 1
    _S.cursor = 0


def before_weight_gemm(w: torch.Tensor,
                       also: Optional[List[torch.Tensor]] = None) -> Optional[List[torch.Tensor]]:
    """Called right before a GEMM whose weight operand is ``w`` (a persistent tensor).  Returns
    the tensors that GEMM should warm (pass them as ``prefetch=`` to :func:`kernels.gemm`): the
    weight of the next weight GEMM of the recorded step order, after ``also`` (tensors this
    layer reads next, e.g. the weight-grad's saved input); None while recording / off."""
    if _S.recording:
        if len(_S.order) < 4096:
            _S.order.append(w)
        return None
    if not _S.armed:
        return None
    i = _S.cursor
    o = _S.order[i] if i < len(_S.order) else None
    if o is None or o.shape != w.shape or o.device != w.device:
        # the GEMM sequence differs from the recorded step: stop, record again from the next
        # step boundary
        _S.armed, _S.order, _S.volatile = False, [], set()
        return None
    if o.data_ptr() != w.data_ptr():
        # a weight operand made per step (a cast of a parameter outside the flat space): the
        # slot stays, never prefetched.  Most slots moving means another model of the same
        # shapes: record again (and drop the old weights)
        _S.volatile.add(i)
        if len(_S.volatile) > len(_S.order) // 2:
            _S.armed, _S.order, _S.volatile = False, [], set()
            return None
    _S.cursor = i + 1
    if not enabled() or not w.is_cuda:
        return None
    nxt = list(also) if also and _MODE != "w0" else []  # ("w0": weights only, for A/Bs)
    if i + 1 < len(_S.order) and i + 1 not in _S.volatile:
        nxt.append(_S.order[i + 1])
    # (a model split over devices: only tensors on this GEMM's device can be warmed by it)
    nxt = [t for t in nxt
           if t is not None and t.device == w.device and t.is_contiguous() and t.numel()]
    return nxt[:2] or None

