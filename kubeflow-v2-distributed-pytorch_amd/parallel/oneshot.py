"""One-shot collectives over HIP IPC peer pointers (SURVEY §5.8 design item 5).

For latency-bound messages — DDP's per-forward BN buffer broadcast (C4: ~38 KB for ResNet-18,
~212 KB for ResNet-50) and tiny gradient buckets — a ring collective's 2(N-1) dependent hops
cost more than the bytes.  Here every rank maps every peer's workspace once (hipIpcGetMemHandle
/ hipIpcOpenMemHandle, handles exchanged over the process group) and ONE kernel per call stages
the message, flags it to the peers over xGMI and reads the peers' copies directly
(csrc/kernels/oneshot.hip): one hop, a deterministic rank-order sum, no host sync, graph-capture
safe (epochs live in device memory).

Scope: the ranks of one node (all peers reachable over xGMI; at most 8), every rank issuing the
same sequence of calls with the same sizes.  DDP uses it for C4 when ``MIPIPE_ONESHOT=1``;
RCCL stays the default (the one-shot path is checked on one GPU with two processes sharing it
— ``tests/test_oneshot_gpu.py`` — not yet on an 8-GPU mesh).

Failure ("a hang becomes an error"): a kernel that waits longer than ``timeout_s``
(``MIPIPE_ONESHOT_TIMEOUT_S``, default 120 s) for a peer records {peer, epoch} in its error words
and leaves the output untouched instead of reading a slot the peer never filled.  :meth:`check`
turns the error words into a :class:`~mipipe.parallel.ddp.CollectiveSequenceError`; it reads
them through an asynchronous copy into pinned memory (no host sync), so DDP can poll it at every
log interval and once, synchronously, at the end of training.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

__all__ = ["OneShotComm", "oneshot_enabled"]


def oneshot_enabled() -> bool:
    return os.environ.get("MIPIPE_ONESHOT", "0") == "1"


def _same_node(group) -> bool:
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    if lw is not None:
        return int(lw) == dist.get_world_size(group)
    import socket
    names = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, socket.gethostname(), group=group)
    return len(set(names)) == 1


class OneShotComm:
    """One workspace per rank with ``cap_bytes`` per message; ``all_reduce`` (fp32, in place,
    sum or average) and ``broadcast`` (any dtype, in place)."""

    def __init__(self, group=None, cap_bytes: int = 1 << 20, device: Optional[torch.device] = None,
                 timeout_s: Optional[float] = None):
        from mipipe.ops._native import native
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world > 8:
            raise ValueError("one-shot collectives span one node (<= 8 xGMI peers)")
        if not _same_node(group):
            raise ValueError("one-shot collectives need every rank on this node")
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        if timeout_s is None:
            timeout_s = float(os.environ.get("MIPIPE_ONESHOT_TIMEOUT_S", "120"))
        self.timeout_s = float(timeout_s)
        self._c = native().OneShot(self.rank, self.world, int(cap_bytes), dev.index,
                                   self.timeout_s)
        hs = [None] * self.world
        dist.all_gather_object(hs, bytes(self._c.handle()), group=group)
        self._c.open(hs)

    @property
    def cap(self) -> int:
        return self._c.cap

    def fits(self, t: torch.Tensor) -> bool:
        nb = t.numel() * t.element_size()
        return (t.is_cuda and t.is_contiguous() and nb % 16 == 0 and nb <= self.cap
                and t.data_ptr() % 16 == 0)

    def all_reduce(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        self._c.all_reduce(t, average)
        return t

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        self._c.broadcast(t, src)
        return t

    def error(self) -> int:
        """1 + the peer a wait gave up on (0: none); synchronises the device."""
        return self._c.error()

    def check(self, final: bool = False) -> None:
        """Raise if any one-shot call so far gave up waiting for a peer.

        ``final=False`` (the per-log-interval poll): reads the error words copied by the previous
        poll if that copy has landed, then requests a new copy — no host synchronisation, so the
        answer lags by one interval.  ``final=True``: synchronous read (end of training)."""
        from mipipe.parallel.ddp import CollectiveSequenceError
        if final:
            peer, epoch = self._c.error_info()
        else:
            if torch.cuda.is_current_stream_capturing():
                return
            peer, epoch = self._c.poll_error()
            self._c.request_error()
        if peer > 0:
            raise CollectiveSequenceError(
                f"one-shot collective: rank {self.rank} waited more than {self.timeout_s:g} s for "
                f"rank {peer - 1} at call epoch {epoch} (that rank skipped or stalled a collective "
                "this rank issued); the result of that call was not written")
