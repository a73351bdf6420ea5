"""HIP-graph capture of a whole training step (forward + backward + optimizer).

The MI355X answer to "launch-bound inner loops": one ResNet-18/CIFAR step is ~225 kernel
launches whose CPU-side dispatch (Python autograd + launch latency) leaves the GPU idle for
~15 % of the step; replaying a captured hipGraph issues the same kernels back to back with one
launch.  Every kernel still runs every step — nothing is cached or skipped.

Constraints of capture (checked or documented):
* static shapes and addresses: the step reads its batch from fixed input tensors; callers either
  copy each batch into them (``GraphedStep.step(x, y)``) or capture one graph per resident
  batch buffer (``GraphedStep(..., inputs=[(x0, y0), (x1, y1)])``, zero copies);
* no host synchronisation inside the step;
* host-side scalars are frozen at capture: SGD has none; AdamW keeps its step count on the
  device and dropout seeds take their per-step part from a device counter (BERT), otherwise
  :func:`graph_safe` refuses the step;
* under mipipe DDP the bucket all-reduces are captured too (RCCL on the process group's
  stream); capture runs in ``thread_local`` error mode so the RCCL watchdog thread can keep
  querying its events, and capture starts only once every process group's watchdog tracks no
  outstanding work (:func:`_drain_collective_watchdog`);
* warm-up and capture run on one stream (:func:`step_stream`), so no parameter's AccumulateGrad
  node is pinned to a stream outside the capture.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch


def graph_safe(model: torch.nn.Module, optimizer) -> Tuple[bool, str]:
    """Whether a step of ``model`` + ``optimizer`` can be replayed from one capture.

    Per-step values must live on the device: SGD has none; AdamW's step count / bias corrections
    are a device counter (``device_step``); mipipe dropout seeds take their per-step part from a
    device counter when the model declares ``device_seeds`` (BERT on the GPU)."""
    from mipipe.optim import SGD, AdamW
    if isinstance(optimizer, AdamW):
        if not getattr(optimizer, "device_step", False):
            return False, "AdamW without a device step counter (CPU) uses host-side bias corrections"
    elif not isinstance(optimizer, SGD):
        return False, f"{type(optimizer).__name__} uses host-side per-step scalars"
    root = getattr(model, "module", model)
    dev_seeds = bool(getattr(root, "device_seeds", False))
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout) and m.p > 0 and m.training:
            return False, "torch.nn.Dropout draws its mask from the host generator state"
        if (getattr(m, "p_hidden", 0) or getattr(m, "p_attn", 0)) and not dev_seeds:
            return False, "dropout seeds are host-side per-step values"
    return True, ""


def _drain_collective_watchdog(timeout_s: float = 60.0) -> None:
    """Block until every process group's watchdog has retired all of its enqueued work.

    Why: ProcessGroupNCCL's watchdog thread polls the end events of every collective it still
    tracks.  An event query that lands while this thread is capturing can fail the capture and
    abort the process (observed once in ~10 world-1 RCCL captures in round 2).  The condition
    that makes capture safe is "the watchdog tracks no work" — ``_wait_for_pending_works()``
    waits for exactly that (the PG's work list and its completed-work list both empty).  The
    device is synchronised before this is called, so every tracked work is complete and is
    retired on the watchdog's next poll; nothing is enqueued during capture itself (captured
    collectives are not handed to the watchdog)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return
    from torch.distributed import distributed_c10d as c10d
    pgs = list(getattr(c10d._world, "pg_map", {}).keys()) or [c10d._get_default_group()]
    for pg in pgs:
        try:
            backend = dist.get_backend(pg)
        except Exception:
            backend = ""
        if "nccl" not in str(backend):
            continue  # gloo / other backends have no event-polling watchdog
        wait = getattr(pg, "_wait_for_pending_works", None)
        if wait is None:
            raise RuntimeError("this torch build has no ProcessGroup._wait_for_pending_works: "
                               "cannot prove the collective watchdog is idle before capture")
        wait()


_STEP_STREAMS = {}


def step_stream(device: torch.device) -> "torch.cuda.Stream":
    """The one side stream every eager warm-up step AND the capture of a device run on.

    Autograd pins each parameter's AccumulateGrad node to the stream current when the node was
    created; a node created on stream A and still alive when backward runs on stream B makes
    the engine synchronise A with B ("AccumulateGrad node's stream does not match ...") — during
    capture that is a cross-stream dependency on a stream outside the capture.  Warm-up and
    capture on the same stream removes the mismatch at its cause."""
    key = (device.type, device.index)
    if key not in _STEP_STREAMS:
        _STEP_STREAMS[key] = torch.cuda.Stream(device)
    return _STEP_STREAMS[key]


class CaptureFailed(RuntimeError):
    """The hipGraph CAPTURE of a step failed (its eager warm-up steps succeeded).  Captured
    collectives never execute during capture, so every rank can still agree to run eagerly;
    an exception from a warm-up step is NOT wrapped: those steps issue real collectives, and a
    rank that failed there must exit instead of joining a fallback protocol its peers are not
    in."""


class GraphedStep:
    """Capture ``step_fn(*batch) -> loss`` into hipGraph(s) after ``warmup`` eager steps.

    ``inputs``: the resident batch buffers (tuples of tensors) to capture against, one graph
    each; when omitted, one graph is captured against internal static copies of ``example`` and
    :meth:`step` copies each batch in."""

    def __init__(self, step_fn: Callable[..., torch.Tensor], example: Sequence[torch.Tensor],
                 warmup: int = 3, inputs: Optional[Sequence[Sequence[torch.Tensor]]] = None):
        self.fn = step_fn
        dev = example[0].device
        self.static: List[Tuple[torch.Tensor, ...]] = (
            [tuple(b) for b in inputs] if inputs is not None
            else [tuple(t.clone() for t in example)])
        self.copy_in = inputs is None
        s = step_stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):  # warm up on the capture stream (allocator + lazy init)
            for i in range(max(1, warmup)):
                batch = self.static[i % len(self.static)]
                self.warmup_loss = self.fn(*batch).detach()  # loss of the last eager step
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        _drain_collective_watchdog()
        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.losses: List[torch.Tensor] = []
        pool = None
        try:
            for batch in self.static:
                g = torch.cuda.CUDAGraph()
                # thread_local: the process group's watchdog thread may still poll its
                # (retired) work events while this thread captures; global mode would fail them
                with torch.cuda.graph(g, pool=pool, stream=s, capture_error_mode="thread_local"):
                    loss = self.fn(*batch).detach()  # drop the autograd graph: no stale nodes
                pool = g.pool()
                self.graphs.append(g)
                self.losses.append(loss)
            torch.cuda.synchronize(dev)
        except Exception as exc:  # noqa: BLE001 — re-raised as the capture-phase failure
            raise CaptureFailed(f"hipGraph capture failed: {exc!r}") from exc

    def replay(self, i: int = 0) -> torch.Tensor:
        """Run one step on resident batch ``i``; returns the (device) loss."""
        k = i % len(self.graphs)
        self.graphs[k].replay()
        return self.losses[k]

    def step(self, *batch: torch.Tensor) -> torch.Tensor:
        """Copy a batch into the static buffers and run one step."""
        if not self.copy_in:
            raise RuntimeError("captured against resident buffers: use replay(i)")
        for dst, src in zip(self.static[0], batch):
            dst.copy_(src, non_blocking=True)
        return self.replay(0)
