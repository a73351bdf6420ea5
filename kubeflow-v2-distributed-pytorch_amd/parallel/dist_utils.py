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


def init_distributed(backend: str, init_method: str, world_size: int, rank: int,
                     timeout_s: float = 1800.0, device: Optional[torch.device] = None) -> None:
    """``dist.init_process_group`` with a finite collective timeout (hang -> error, §5.3).
    ``nccl`` (= RCCL) needs GPUs; without one the backend falls back to gloo."""
    if backend == "nccl" and not torch.cuda.is_available():
        backend = "gloo"
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    kw = {}
    if device is not None and backend == "nccl":
        kw["device_id"] = device
    dist.init_process_group(backend=backend, init_method=init_method, world_size=world_size,
                            rank=rank, timeout=datetime.timedelta(seconds=timeout_s), **kw)


def cleanup() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
