"""The one environment builder behind every mipipe launcher (the rank-process env contract).

Both entry points start ranks through :func:`rank_env`: ``launch.launcher.build_envs`` (the
aiplatform ``CustomTrainingJob`` replicas, reference nb:181-188) and ``launch.local.rank_envs``
(``bench.py --gpus N``, torchrun-style).  GPU visibility policy on one xGMI node — two modes:

* ``"slice"`` (the launcher's default whenever a replica owns fewer GPUs than the node exposes):
  each replica SEES only its own GPUs (``HIP_VISIBLE_DEVICES`` narrowed, offset 0 — or
  ``ROCR_VISIBLE_DEVICES`` when that is where the ids came from), exactly what
  a Vertex VM with ``accelerator_count`` GPUs looks like.  Programs that count devices —
  the unmodified reference task.py (``ngpus_per_node = torch.cuda.device_count()``, task.py:102)
  or a non-distributed ``DataParallel(model)`` (task.py:201-208) — then stay on their slice.
* ``"all"`` (opt-in, for mipipe-aware programs): every rank sees ALL GPUs the launcher may hand
  out and OWNS a slice: its device is ``cuda:(MIPIPE_DEVICE_OFFSET + local index)``, where the
  local index is ``LOCAL_RANK`` (torchrun mode) or the ``mp.spawn`` child index (the reference's
  ``--multiprocessing-distributed`` mode, task.py:117-124).  RCCL maps peer buffers over xGMI
  (P2P/IPC) only between devices a process can see, so this keeps cross-replica traffic on
  xGMI instead of the host shared-memory transport.  Every mipipe consumer (train/task.py,
  parallel/data_parallel.py, bench.py) honours the offset and ``MIPIPE_LOCAL_GPUS``.

In both modes ``MIPIPE_LOCAL_GPUS`` is the number of GPUs of the replica (what task.py counts as
``ngpus_per_node``).  A replica with no accelerators runs on the CPU (``MIPIPE_FORCE_CPU=1``, no
visible GPU).
"""
from __future__ import annotations

import os
from typing import Dict, Mapping, Optional

__all__ = ["rank_env", "device_offset", "local_gpus", "local_device_ids"]


def device_offset(env: Optional[Mapping[str, str]] = None) -> int:
    env = os.environ if env is None else env
    return int(env.get("MIPIPE_DEVICE_OFFSET", "0") or 0)


def local_gpus(env: Optional[Mapping[str, str]] = None) -> Optional[int]:
    """GPUs of this replica (``MIPIPE_LOCAL_GPUS``), or None when the launcher did not say."""
    env = os.environ if env is None else env
    v = env.get("MIPIPE_LOCAL_GPUS")
    return int(v) if v not in (None, "") else None


def local_device_ids(env: Optional[Mapping[str, str]] = None) -> Optional[list]:
    """CUDA device indices this replica owns ([offset, offset + MIPIPE_LOCAL_GPUS)), or None
    when no launcher said (then: every visible device)."""
    n = local_gpus(env)
    if n is None:
        return None
    off = device_offset(env)
    return list(range(off, off + n))


def rank_env(base: Mapping[str, str], *, master_addr: str, master_port: int,
             world: Optional[int] = None, rank: Optional[int] = None,
             local_rank: Optional[int] = None, local_world: Optional[int] = None,
             group_rank: Optional[int] = None, gpu_offset: int = 0,
             replica_gpus: Optional[int] = None, extra: Optional[Mapping[str, str]] = None,
             rccl: bool = True, visible: Optional[str] = None,
             visible_var: str = "HIP_VISIBLE_DEVICES") -> Dict[str, str]:
    """Environment of one launched process.  ``replica_gpus``: GPUs owned by this process's
    replica (None: leave the GPU variables alone; 0: CPU-only replica).  ``visible``: the
    replica's own GPU ids ("slice" mode: HIP_VISIBLE_DEVICES narrowed to them, offset 0), or
    None ("all" mode: visibility left as found, the slice named by the offset).  ``visible_var``:
    the variable the ids were read from — ``ROCR_VISIBLE_DEVICES`` ids are physical indices,
    so that slice narrows ROCR itself (HIP would renumber them relative to the ROCR set)."""
    e = dict(base)
    if extra:
        e.update(extra)
    if rccl:
        from mipipe.parallel.dist_utils import configure_rccl_env
        configure_rccl_env(e)  # high-priority comm stream + MIPIPE_RCCL_PROFILE channels
    e["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"  # dmabuf IPC: the only mode the host driver supports
    e["MASTER_ADDR"] = master_addr
    e["MASTER_PORT"] = str(master_port)
    for k, v in (("WORLD_SIZE", world), ("RANK", rank), ("LOCAL_RANK", local_rank),
                 ("LOCAL_WORLD_SIZE", local_world), ("GROUP_RANK", group_rank)):
        if v is not None:
            e[k] = str(v)
    if replica_gpus is not None:
        if replica_gpus == 0:
            e["HIP_VISIBLE_DEVICES"] = ""
            e["MIPIPE_FORCE_CPU"] = "1"
            e.pop("MIPIPE_DEVICE_OFFSET", None)
            e.pop("MIPIPE_LOCAL_GPUS", None)
        else:
            e.pop("MIPIPE_FORCE_CPU", None)
            if visible is not None:
                if visible_var == "ROCR_VISIBLE_DEVICES":
                    e["ROCR_VISIBLE_DEVICES"] = visible
                    e.pop("HIP_VISIBLE_DEVICES", None)
                else:
                    e["HIP_VISIBLE_DEVICES"] = visible
                e.pop("CUDA_VISIBLE_DEVICES", None)
                e["MIPIPE_DEVICE_OFFSET"] = "0"
            else:
                e["MIPIPE_DEVICE_OFFSET"] = str(gpu_offset)
            e["MIPIPE_LOCAL_GPUS"] = str(replica_gpus)
    return e
