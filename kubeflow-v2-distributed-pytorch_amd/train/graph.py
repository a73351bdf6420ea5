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
* host-side scalars are frozen at capture: fine for SGD (momentum buffers are on the device),
  NOT for AdamW's bias correction or per-step dropout seeds — :func:`graph_safe` refuses those;
* under mipipe DDP the bucket all-reduces are captured too (RCCL on the process group's
  stream); capture runs in ``thread_local`` error mode so the RCCL watchdog thread can keep
  querying its events.
"""
from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import torch


def graph_safe(model: torch.nn.Module, optimizer) -> Tuple[bool, str]:
    """Whether a step of ``model`` + ``optimizer`` can be replayed from one capture."""
    from mipipe.optim import SGD
    if not isinstance(optimizer, SGD):
        return False, f"{type(optimizer).__name__} uses host-side per-step scalars"
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout) and m.p > 0 and m.training:
            return False, "dropout seeds are host-side per-step values"
        if getattr(m, "p_hidden", 0) or getattr(m, "p_attn", 0):
            return False, "dropout seeds are host-side per-step values"
    return True, ""


def _drain_collective_watchdog(wait_s: float = 0.5) -> None:
    """Let the process group's watchdog thread retire the (completed) work of the eager warm-up
    collectives before capture starts: it polls every ~100 ms with event queries, and a query
    that lands inside the capture window can fail and abort the process (seen once in ~10
    world-1 RCCL captures, tests/test_ddp_gpu.py).  The device is idle here, so every pending
    work object completes on its next poll."""
    import time
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        time.sleep(wait_s)


class GraphedStep:
    """Capture ``step_fn(x, y) -> loss`` into hipGraph(s) after ``warmup`` eager steps.

    ``inputs``: the resident batch buffers to capture against (one graph each); when omitted,
    one graph is captured against internal static buffers and :meth:`step` copies in."""

    def __init__(self, step_fn: Callable[[torch.Tensor, torch.Tensor], torch.Tensor],
                 example: Tuple[torch.Tensor, torch.Tensor], warmup: int = 3,
                 inputs: Optional[Sequence[Tuple[torch.Tensor, torch.Tensor]]] = None):
        self.fn = step_fn
        dev = example[0].device
        self.static: List[Tuple[torch.Tensor, torch.Tensor]] = (
            list(inputs) if inputs is not None
            else [(example[0].clone(), example[1].clone())])
        self.copy_in = inputs is None
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):  # warm up on a side stream (allocator + lazy init)
            for i in range(max(1, warmup)):
                x, y = self.static[i % len(self.static)]
                self.warmup_loss = self.fn(x, y).detach()  # loss of the last eager step
        torch.cuda.current_stream(dev).wait_stream(s)
        torch.cuda.synchronize(dev)
        _drain_collective_watchdog()
        self.graphs: List[torch.cuda.CUDAGraph] = []
        self.losses: List[torch.Tensor] = []
        pool = None
        for x, y in self.static:
            g = torch.cuda.CUDAGraph()
            # thread_local: the process group's watchdog thread keeps polling its RCCL work
            # events while this thread captures; global mode would fail those queries
            with torch.cuda.graph(g, pool=pool, capture_error_mode="thread_local"):
                loss = self.fn(x, y).detach()  # drop the autograd graph: no stale grad nodes
            pool = g.pool()
            self.graphs.append(g)
            self.losses.append(loss)
        torch.cuda.synchronize(dev)

    def replay(self, i: int = 0) -> torch.Tensor:
        """Run one step on resident batch ``i``; returns the (device) loss."""
        k = i % len(self.graphs)
        self.graphs[k].replay()
        return self.losses[k]

    def step(self, x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
        """Copy a batch into the static buffers and run one step."""
        if not self.copy_in:
            raise RuntimeError("captured against resident buffers: use replay(i)")
        sx, sy = self.static[0]
        sx.copy_(x, non_blocking=True)
        sy.copy_(y, non_blocking=True)
        return self.replay(0)
