"""Rank / world-size helpers and the reference's rendezvous arithmetic.

task.py semantics: ``--world-size`` counts *nodes* (replicas); with
``--multiprocessing-distributed`` the global world is ``nodes * ngpus_per_node``
(task.py:120) and the global rank ``node_rank * ngpus_per_node + local_gpu`` (task.py:146).
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

__all__ = ["global_world_size", "global_rank", "init_distributed", "is_main", "barrier",
           "get_rank", "get_world_size", "cleanup"]


def global_world_size(nodes: int, ngpus_per_node: int) -> int:
    return nodes * ngpus_per_node


def global_rank(node_rank: int, ngpus_per_node: int, local_gpu: int) -> int:
    return node_rank * ngpus_per_node + local_gpu


def get_rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def get_world_size() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def is_main() -> bool:
    return get_rank() == 0


def barrier(device: Optional[torch.device] = None) -> None:
    if dist.is_available() and dist.is_initialized():
        if device is not None and device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


# RCCL / ProcessGroupNCCL settings for the MI355X node, applied (as defaults: the environment
# wins) before any process group exists.  Each one is measured, not folklore:
#  * TORCH_NCCL_HIGH_PRIORITY=1 — the PG's communication stream becomes a high-priority HIP
#    stream.  Measured on one MI355X (tools/r3/overlap_probe.py, profiles/r3_overlap_probe.txt):
#    a 256 MB RCCL all-reduce issued beside 40 back-to-back conv kernels overlapped them 0.08-0.13
#    of its duration eagerly at normal priority and 0.84 at high priority (hipGraph replay: 0.78-
#    0.91 either way).  Without it an eager DDP step serialises its bucket all-reduces behind the
#    backward kernels already queued — the round-2 trace's "0.0 % overlapped".
#  * HSA_ENABLE_IPC_MODE_LEGACY=0 — this host's driver only supports dmabuf IPC; RCCL's P2P
#    buffers (xGMI peers) fail to map without it.
RCCL_ENV_DEFAULTS = {
    "TORCH_NCCL_HIGH_PRIORITY": "1",
    "HSA_ENABLE_IPC_MODE_LEGACY": "0",
}


def configure_rccl_env(env: Optional[dict] = None) -> dict:
    """Apply :data:`RCCL_ENV_DEFAULTS` to ``env`` (``os.environ`` by default) without
    overriding values already set; returns the target mapping."""
    target = os.environ if env is None else env
    for k, v in RCCL_ENV_DEFAULTS.items():
        target.setdefault(k, v)
    return target


def init_distributed(backend: str, init_method: str, world_size: int, rank: int,
                     timeout_s: float = 1800.0, device: Optional[torch.device] = None) -> None:
    """``dist.init_process_group`` with a finite collective timeout (hang -> error, §5.3).
    ``nccl`` (= RCCL) needs GPUs; without one the backend falls back to gloo."""
    if backend == "nccl" and not torch.cuda.is_available():
        backend = "gloo"
    configure_rccl_env()
    kw = {}
    if device is not None and backend == "nccl":
        kw["device_id"] = device
    dist.init_process_group(backend=backend, init_method=init_method, world_size=world_size,
                            rank=rank, timeout=datetime.timedelta(seconds=timeout_s), **kw)


def cleanup() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
