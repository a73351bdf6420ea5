"""Single-process multi-GPU data parallelism (reference path (d), task.py:201-208).

The reference wraps the model in ``torch.nn.DataParallel`` when neither a process group nor a
GPU index is given (``/root/reference/task.py:201-208``; dead in practice, SURVEY §2.3, but part
of the API surface).  This is mipipe's own implementation, built around the flat parameter
space (:mod:`mipipe.optim.flat`) instead of torch's per-forward ``replicate``:

* **persistent replicas** — device ``i > 0`` gets a deep copy of the module, built once, with
  its *own* flat fp32 parameter / gradient / bf16-shadow buffers laid out exactly like the
  master's.  The HIP kernels of a replica therefore read their compute-dtype weights and write
  their weight gradients straight into device-local flat buffers, as on one GPU;
* **one collective per buffer per step** — before each forward the master's flat parameters
  and shadow (plus module buffers) are broadcast to every replica, and at the end of backward
  every replica's flat gradient is summed into the master's.  With distinct CUDA devices both
  run as in-process RCCL collectives (``torch.cuda.nccl`` over one communicator clique — ring
  broadcast / reduce across the xGMI links, not 7 serial peer copies into GPU 0); otherwise a
  pairwise tree of copy+add;
* **scatter / threaded apply / gather** — the batch is split along ``dim`` into one chunk per
  device, each replica runs in its own host thread under its device (kernels go to that
  device's current stream), and outputs are concatenated on ``output_device``.  Chunk copies
  and the gather are differentiable, so backward fans out to every replica; an identity node
  on the gathered output queues the gradient reduction as an autograd-engine callback, which
  runs once all devices' backward work has been issued.

As in torch's DataParallel, BatchNorm statistics are per chunk and only the master's running
statistics survive (replica buffers are overwritten by the next broadcast).  Device lists may
repeat a device or name ``"cpu"`` (replicas then share a device): the CPU tests and the 1-GPU
box exercise the full replicate/apply/reduce logic that way.  With one device it is a plain
pass-through.
"""
from __future__ import annotations

import copy
import threading
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as tnn

from mipipe.optim.flat import FlatParamSpace, flat_space_for

__all__ = ["DataParallel"]


def _as_device(d) -> torch.device:
    if isinstance(d, torch.device):
        return d
    if isinstance(d, int):
        return torch.device("cuda", d)
    return torch.device(d)


def _distinct_cuda(devs: Sequence[torch.device]) -> bool:
    idx = [d.index for d in devs]
    return all(d.type == "cuda" for d in devs) and len(set(idx)) == len(idx)


def _device_ctx(dev: torch.device):
    if dev.type == "cuda":
        return torch.cuda.device(dev)
    import contextlib
    return contextlib.nullcontext()


def _nccl_ok(tensors: List[torch.Tensor]) -> bool:
    if not _distinct_cuda([t.device for t in tensors]):
        return False
    try:
        import torch.cuda.nccl as nccl
        return nccl.is_available(tensors)
    except Exception:
        return False


def _broadcast_into(src: torch.Tensor, dsts: List[torch.Tensor]) -> None:
    """Copy ``src`` into every tensor of ``dsts`` (same shape; one per device)."""
    if not dsts:
        return
    group = [src] + dsts
    if _nccl_ok(group):
        import torch.cuda.nccl as nccl
        nccl.broadcast(group, root=0)
        return
    for d in dsts:
        d.copy_(src, non_blocking=True)


def _reduce_into(dst: torch.Tensor, srcs: List[torch.Tensor]) -> None:
    """``dst += sum(srcs)`` (same shape; srcs may live on other devices)."""
    if not srcs:
        return
    group = [dst] + srcs
    if _nccl_ok(group):
        import torch.cuda.nccl as nccl
        nccl.reduce(group, root=0)  # in place into dst
        return
    # pairwise tree: round r adds slot i+2^r into slot i, so 8 devices take 3 rounds
    # and the copies of one round run over disjoint links
    slots = list(group)
    step = 1
    while step < len(slots):
        for i in range(0, len(slots) - step, 2 * step):
            a, b = slots[i], slots[i + step]
            if i == 0:
                a.add_(b.to(a.device, non_blocking=True))
            else:  # intermediate sums must not alias a replica's gradient buffer
                slots[i] = a + b.to(a.device, non_blocking=True)
        step *= 2


class _QueueReduce(torch.autograd.Function):
    """Identity whose backward schedules the replica-gradient reduction for the end of the
    current backward pass (after every device's backward has been issued)."""

    @staticmethod
    def forward(ctx, dp: "DataParallel", x: torch.Tensor) -> torch.Tensor:
        ctx.dp = dp
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        dp = ctx.dp
        if not dp._reduce_queued:
            dp._reduce_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(dp._reduce_grads)
        return None, g


def _split(obj, n: int, dim: int):
    """Per-device chunks of a (nested) argument; ``None`` count = not a tensor."""
    if isinstance(obj, torch.Tensor):
        return list(obj.chunk(n, dim))
    if isinstance(obj, (list, tuple)) and obj:
        parts = [_split(o, n, dim) for o in obj]
        k = min(len(p) for p in parts if isinstance(p, list)) if any(isinstance(p, list) for p in parts) else None
        if k is None:
            return obj
        return [type(obj)(p[i] if isinstance(p, list) else p for p in parts) for i in range(k)]
    if isinstance(obj, dict) and obj:
        parts = {key: _split(v, n, dim) for key, v in obj.items()}
        lists = [p for p in parts.values() if isinstance(p, list)]
        if not lists:
            return obj
        k = min(len(p) for p in lists)
        return [{key: (p[i] if isinstance(p, list) else p) for key, p in parts.items()} for i in range(k)]
    return obj


def _to(obj, dev: torch.device):
    if isinstance(obj, torch.Tensor):
        return obj if obj.device == dev else obj.to(dev, non_blocking=True)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to(o, dev) for o in obj)
    if isinstance(obj, dict):
        return {k: _to(v, dev) for k, v in obj.items()}
    return obj


def _gather(outs: List[Any], dev: torch.device, dim: int):
    first = outs[0]
    if isinstance(first, torch.Tensor):
        if first.dim() == 0:  # per-replica scalars (e.g. a loss): stacked, like torch's DP
            return torch.stack([o.to(dev) for o in outs])
        return torch.cat([o.to(dev) for o in outs], dim)
    if isinstance(first, (list, tuple)):
        return type(first)(_gather([o[i] for o in outs], dev, dim) for i in range(len(first)))
    if isinstance(first, dict):
        return {k: _gather([o[k] for o in outs], dev, dim) for k in first}
    return first


def _map_tensors(obj, fn):
    if isinstance(obj, torch.Tensor):
        return fn(obj)
    if isinstance(obj, (list, tuple)):
        return type(obj)(_map_tensors(o, fn) for o in obj)
    if isinstance(obj, dict):
        return {k: _map_tensors(v, fn) for k, v in obj.items()}
    return obj


class DataParallel(tnn.Module):
    """``torch.nn.DataParallel``-compatible wrapper (``module``, ``device_ids``,
    ``output_device``, ``dim``; state_dict keys ``module.*``)."""

    def __init__(self, module: tnn.Module, device_ids: Optional[Sequence] = None,
                 output_device=None, dim: int = 0):
        super().__init__()
        self.module = module
        self.dim = dim
        if device_ids is None:
            # the replica's own GPUs when a launcher named a slice (launch/env.py), else every
            # visible device (torch.nn.DataParallel's default, task.py:204)
            from mipipe.launch.env import local_device_ids
            device_ids = local_device_ids()
            if device_ids is None:
                device_ids = (list(range(torch.cuda.device_count())) if torch.cuda.is_available()
                              else [])
        self.device_ids = list(device_ids)
        self.devices: List[torch.device] = [_as_device(d) for d in self.device_ids]
        self.output_device = (_as_device(output_device) if output_device is not None
                              else (self.devices[0] if self.devices else None))
        # replicas are NOT registered submodules: parameters()/state_dict() see the master only
        self.__dict__["_replicas"]: List[tnn.Module] = []
        self.__dict__["_rep_spaces"]: List[Optional[FlatParamSpace]] = []
        self.__dict__["_rep_params"]: List[List[tnn.Parameter]] = []
        self._master_space: Optional[FlatParamSpace] = None
        self._active = 1
        self._reduce_queued = False

    # ------------------------------------------------------------------ replicas
    def _build_replicas(self, space: Optional[FlatParamSpace]) -> None:
        mparams = list(self.module.parameters())
        self._replicas.clear()
        self._rep_spaces.clear()
        self._rep_params.clear()
        for dev in self.devices[1:]:
            rep = copy.deepcopy(self.module).to(dev)
            for m in rep.modules():  # per-device caches (kernel workspaces, shadow views)
                for k in [k for k in m.__dict__ if k.startswith("_mipipe_") or k == "_shadow"]:
                    del m.__dict__[k]
            rparams = list(rep.parameters())
            for pm, pr in zip(mparams, rparams):
                pr.__dict__.update({k: v for k, v in pm.__dict__.items() if k.startswith("_mipipe")})
                pr.grad = None
            rs = None
            if space is not None:
                index = {id(p): i for i, p in enumerate(mparams)}
                rs = FlatParamSpace([rparams[index[id(p)]] for p in space.params], space.shadow_dtype)
                if rs.numel != space.numel or len(rs.offsets) != len(space.offsets):
                    raise RuntimeError("replica flat layout differs from the master's")
                rs.bind_modules(rep)
            self._replicas.append(rep)
            self._rep_spaces.append(rs)
            self._rep_params.append(rparams)
        self._master_space = space

    def _sync(self, n: int) -> List[tnn.Module]:
        mparams = list(self.module.parameters())
        space = flat_space_for(mparams[0]) if mparams else None
        if space is not None and not space.owns(p for p in mparams if p.requires_grad):
            space = None
        if len(self._replicas) != len(self.devices) - 1 or space is not self._master_space:
            self._build_replicas(space)
        reps = self._replicas[: n - 1]
        with torch.no_grad():
            if space is not None:
                space.sync_shadow()
                _broadcast_into(space.flat, [rs.flat for rs in self._rep_spaces[: n - 1]])
                if space.shadow is not None:
                    _broadcast_into(space.shadow, [rs.shadow for rs in self._rep_spaces[: n - 1]])
                for rs in self._rep_spaces[: n - 1]:
                    rs.mark_synced()
                frozen = [i for i, p in enumerate(mparams) if not p.requires_grad]
            else:
                frozen = range(len(mparams))
            for i in frozen:
                _broadcast_into(mparams[i].data, [rp[i].data for rp in self._rep_params[: n - 1]])
            rbufs = [list(r.buffers()) for r in reps]
            for j, b in enumerate(self.module.buffers()):
                _broadcast_into(b, [rb[j] for rb in rbufs])
        return [self.module] + reps

    def _reduce_grads(self) -> None:
        self._reduce_queued = False
        n = self._active
        space = self._master_space
        with torch.no_grad():
            if space is not None:
                srcs = [rs.flat_grad for rs in self._rep_spaces[: n - 1]]
                _reduce_into(space.flat_grad, srcs)
                for rs in self._rep_spaces[: n - 1]:
                    rs.flat_grad.zero_()
                return
            for i, pm in enumerate(self.module.parameters()):
                gs = [rp[i].grad for rp in self._rep_params[: n - 1] if rp[i].grad is not None]
                if not gs:
                    continue
                if pm.grad is None:
                    pm.grad = torch.zeros_like(pm)
                _reduce_into(pm.grad, gs)
                for rp in self._rep_params[: n - 1]:
                    rp[i].grad = None

    # ------------------------------------------------------------------ forward
    def forward(self, *inputs, **kwargs):
        if len(self.devices) <= 1:
            return self.module(*inputs, **kwargs)
        nd = len(self.devices)
        pieces = _split((inputs, kwargs), nd, self.dim)
        if not isinstance(pieces, list):  # nothing to split: run on the master only
            return self.module(*inputs, **kwargs)
        n = len(pieces)
        replicas = self._sync(n)
        self._active = n
        devs = self.devices[:n]
        results: List[Any] = [None] * n
        errors: List[Optional[BaseException]] = [None] * n
        grad_on = torch.is_grad_enabled()
        autocast = torch.is_autocast_enabled("cuda")
        # autocast state is thread-local: hand the caller's dtype to every worker thread, or the
        # replicas on other devices would fall back to autocast's default (fp16)
        ac_dtype = torch.get_autocast_dtype("cuda")
        # a backward that raised before its final callbacks ran left the flag set: every later
        # backward would skip the replica-gradient reduction
        self._reduce_queued = False

        def run(i: int) -> None:
            try:
                with _device_ctx(devs[i]), torch.set_grad_enabled(grad_on), \
                        torch.autocast("cuda", dtype=ac_dtype, enabled=autocast) if devs[i].type == "cuda" else _nullctx():
                    a, kw = _to(pieces[i], devs[i])
                    results[i] = replicas[i](*a, **kw)
            except BaseException as e:  # re-raised on the caller's thread
                errors[i] = e

        threads = [threading.Thread(target=run, args=(i,)) for i in range(1, n)]
        for t in threads:
            t.start()
        run(0)
        for t in threads:
            t.join()
        for e in errors:
            if e is not None:
                raise e
        out = _gather(results, self.output_device, self.dim)
        if grad_on and n > 1:
            def hook(t: torch.Tensor) -> torch.Tensor:
                if t.requires_grad and t.is_floating_point():
                    return _QueueReduce.apply(self, t)
                return t
            out = _map_tensors(out, hook)
        return out


def _nullctx():
    import contextlib
    return contextlib.nullcontext()
