"""Flat parameter / gradient / shadow storage shared by the optimizer and the DDP reducer.

All parameters of a model live in ONE fp32 buffer, all gradients in ONE fp32 buffer and the
compute-dtype (bf16) weight shadows in ONE buffer, each parameter being a view at the same
offset in all three.  Consequences on MI355X:

* the optimizer step is a single memory-bound HIP kernel over the whole model (SGD: reads
  p, g, m; writes p, m and the bf16 shadow) instead of ~160 per-tensor launches;
* gradient buckets for the all-reduce are contiguous slices of the gradient buffer, so RCCL
  reduces them in place (no pack/unpack copies) — buffers are laid out in *reverse*
  registration order, the order autograd produces gradients (parameters tagged
  ``_mipipe_flat_first`` first: ready at the start of the backward);
* ``zero_grad`` is one memset; the bf16 shadow the kernels read is refreshed by the optimizer
  kernel itself, so no per-layer weight cast runs in the forward.

Offsets are aligned to 64 elements (256 B) so every view starts on a 16-byte boundary for
vectorised kernel access.

A parameter tagged ``p._mipipe_pad_rows = R`` (R > p.shape[0]) gets R rows reserved: the extra
rows are zeros in all three buffers (no gradient ever lands there, so the optimizer keeps them
zero), and :meth:`FlatParamSpace.padded_view` exposes the [R, ...] view — e.g. a vocabulary
embedding used as the tied MLM decoder, padded to the GEMM tile width without a per-step copy.
"""
from __future__ import annotations

import weakref
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.nn as tnn

__all__ = ["FlatParamSpace", "get_flat_space", "flat_space_for"]

_ALIGN = 64
_REGISTRY: "weakref.WeakValueDictionary[int, FlatParamSpace]" = weakref.WeakValueDictionary()


def _dense_strides_ok(p: torch.Tensor) -> bool:
    return p.is_contiguous() or (p.dim() == 4 and p.is_contiguous(memory_format=torch.channels_last))


def _view(buf: torch.Tensor, off: int, like: torch.Tensor) -> torch.Tensor:
    return buf.as_strided(like.shape, like.stride(), buf.storage_offset() + off)


def _pad_rows(p: torch.Tensor) -> Optional[int]:
    r = getattr(p, "_mipipe_pad_rows", None)
    if r is None or p.dim() == 0 or r <= p.shape[0] or not p.is_contiguous():
        return None
    return int(r)


def _reserved(p: torch.Tensor) -> int:
    r = _pad_rows(p)
    n = p.numel() if r is None else r * (p.numel() // p.shape[0])
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


class FlatParamSpace:
    def __init__(self, params: Iterable[tnn.Parameter], shadow_dtype: Optional[torch.dtype] = None):
        self.params: List[tnn.Parameter] = [p for p in params]
        if not self.params:
            raise ValueError("no parameters")
        dev = self.params[0].device
        for p in self.params:
            if p.device != dev:
                raise ValueError("all parameters must be on one device")
            if p.dtype != torch.float32:
                raise ValueError(f"master parameters must be fp32, got {p.dtype}")
            if not _dense_strides_ok(p):
                p.data = p.data.contiguous()
        order = list(reversed(self.params))  # gradient-ready order
        # a parameter tagged ``_mipipe_flat_first`` becomes ready at the START of the backward
        # although it was registered first (BERT's tied word embedding: its dense gradient is
        # complete once the MLM decoder's weight-grad ran): it goes to the front
        first = [p for p in order if getattr(p, "_mipipe_flat_first", False)]
        if first:
            order = first + [p for p in order if not getattr(p, "_mipipe_flat_first", False)]
        self.offsets: Dict[int, int] = {}
        off = 0
        for p in order:
            self.offsets[id(p)] = off
            off += _reserved(p)
        self.numel = off
        self.device = dev
        self.flat = torch.zeros(off, dtype=torch.float32, device=dev)
        self.flat_grad = torch.zeros(off, dtype=torch.float32, device=dev)
        self.shadow_dtype = shadow_dtype if shadow_dtype not in (None, torch.float32) else None
        self.shadow = (torch.zeros(off, dtype=self.shadow_dtype, device=dev)
                       if self.shadow_dtype is not None else None)
        self.order = order
        for p in order:
            o = self.offsets[id(p)]
            v = _view(self.flat, o, p)
            v.copy_(p.data)
            p.data = v
            p.grad = _view(self.flat_grad, o, p)
            _REGISTRY[id(p)] = self
        self._synced_version = -1
        self.refresh_shadow()
        from mipipe.ops import prefetch  # a new model: its GEMM weight order is recorded anew
        prefetch.reset()
        self._bound_modules: List[weakref.ref] = []
        self._ready_listeners: List = []

    # ------------------------------------------------------------------ readiness
    def add_ready_listener(self, fn) -> None:
        """``fn(param)`` is called when a kernel wrote a parameter's gradient directly into the
        flat buffer (bypassing autograd's AccumulateGrad and its post-accumulate hooks)."""
        self._ready_listeners.append(fn)

    def grad_ready(self, p: torch.Tensor) -> None:
        for fn in self._ready_listeners:
            fn(p)

    # ------------------------------------------------------------------ views
    def offset(self, p: torch.Tensor) -> int:
        return self.offsets[id(p)]

    def grad_view(self, p: torch.Tensor) -> torch.Tensor:
        return _view(self.flat_grad, self.offsets[id(p)], p)

    def shadow_view(self, p: torch.Tensor) -> Optional[torch.Tensor]:
        if self.shadow is None:
            return None
        return _view(self.shadow, self.offsets[id(p)], p)

    def padded_rows(self, p: torch.Tensor) -> Optional[int]:
        """Rows reserved for ``p`` when it was registered padded (``_mipipe_pad_rows``)."""
        return _pad_rows(p) if id(p) in self.offsets else None

    def padded_view(self, buf: torch.Tensor, p: torch.Tensor) -> torch.Tensor:
        """[padded_rows, *p.shape[1:]] view of ``p``'s slot in ``buf`` (flat / flat_grad /
        shadow); rows beyond p.shape[0] are the reserved zeros."""
        r = self.padded_rows(p)
        if r is None:
            raise ValueError("parameter was not registered with padded rows")
        o = self.offsets[id(p)]
        n = r * (p.numel() // p.shape[0])
        return buf[o: o + n].view(r, *p.shape[1:])

    def ranges(self) -> List[Tuple[int, int, tnn.Parameter]]:
        """(start, end_aligned, param) in flat order."""
        out = []
        for p in self.order:
            o = self.offsets[id(p)]
            out.append((o, o + _reserved(p), p))
        return out

    # ------------------------------------------------------------------ maintenance
    def ensure_grad_views(self) -> None:
        """Re-attach gradient views if user code replaced/cleared ``p.grad``."""
        for p in self.order:
            g = p.grad
            if g is None or g.data_ptr() != self.flat_grad.data_ptr() + 4 * self.offsets[id(p)]:
                if g is not None:
                    self.grad_view(p).copy_(g)
                else:
                    self.grad_view(p).zero_()
                p.grad = self.grad_view(p)

    def zero_grad(self) -> None:
        from mipipe.ops import prefetch  # a step starts: GEMM operand prefetch (ops/prefetch.py)
        prefetch.step_boundary()
        self.flat_grad.zero_()
        self.ensure_grad_views()

    def refresh_shadow(self) -> None:
        if self.shadow is not None:
            self.shadow.copy_(self.flat)
        self.mark_synced()

    def mark_synced(self) -> None:
        """Record parameter versions after params *and* shadow were rewritten together
        (optimizer step, refresh).  HIP kernels writing through raw pointers bump nothing."""
        self._synced_version = self.flat._version
        self._pver = {id(p): p._version for p in self.order}

    def sync_shadow(self, p: Optional[torch.Tensor] = None) -> None:
        """Refresh the shadow if parameters changed through torch ops since the last sync:
        in-place ops on the flat buffer (DDP broadcast) bump ``flat._version``; in-place ops
        on a parameter (``load_state_dict``) bump that parameter's own counter."""
        if self.shadow is None:
            return
        stale = self.flat._version != self._synced_version
        if not stale and p is not None:
            stale = p._version != self._pver.get(id(p), -1)
        if stale:
            self.refresh_shadow()

    def bind_modules(self, root: tnn.Module) -> None:
        """Point every shadow-reading layer of ``root`` at its slice of the shadow buffer."""
        from mipipe.nn import ShadowMixin
        for m in root.modules():
            if isinstance(m, ShadowMixin) and getattr(m, "weight", None) is not None \
                    and id(m.weight) in self.offsets and self.shadow is not None:
                sv = m.operand_view(self.shadow_view(m.weight))
                m.set_shadow(sv if sv.is_contiguous() else None)
        if not any(r() is root for r in self._bound_modules):
            self._bound_modules.append(weakref.ref(root))
            root.register_load_state_dict_post_hook(lambda mod, keys: self.refresh_shadow())

    def owns(self, params: Iterable[torch.Tensor]) -> bool:
        return all(id(p) in self.offsets for p in params)


def flat_space_for(p: torch.Tensor) -> Optional[FlatParamSpace]:
    return _REGISTRY.get(id(p))


def get_flat_space(params: Iterable[tnn.Parameter], shadow_dtype: Optional[torch.dtype] = None,
                   module: Optional[tnn.Module] = None) -> FlatParamSpace:
    """Return the space that already holds exactly these params, or build one."""
    params = [p for p in params if p.requires_grad]
    spaces = {id(s): s for s in (flat_space_for(p) for p in params) if s is not None}
    if len(spaces) == 1:
        s = next(iter(spaces.values()))
        if len(s.params) == len(params):
            if module is not None:
                s.bind_modules(module)
            return s
    if spaces:
        raise RuntimeError("parameters already belong to a different flat space")
    s = FlatParamSpace(params, shadow_dtype)
    if module is not None:
        s.bind_modules(module)
    return s
