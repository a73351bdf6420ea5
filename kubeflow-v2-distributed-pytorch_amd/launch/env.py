"""The one environment builder behind every mipipe launcher (the rank-process env contract).

Both entry points start ranks through :func:`rank_env`: ``launch.launcher.build_envs`` (the
aiplatform ``CustomTrainingJob`` replicas, reference nb:181-188) and ``launch.local.rank_envs``
(``bench.py --gpus N``, torchrun-style).  GPU visibility policy on one xGMI node:

* every rank sees ALL GPUs the launcher may hand out (``HIP_VISIBLE_DEVICES`` is left as the
  launcher found it).  RCCL maps peer buffers over xGMI (P2P/IPC) only between devices a
  process can see; hiding peers forces the shared-memory transport through the host.
* a rank's own device is ``cuda:(MIPIPE_DEVICE_OFFSET + local index)``, where the local index is
  ``LOCAL_RANK`` (torchrun mode) or the ``mp.spawn`` child index (the reference's
  ``--multiprocessing-distributed`` mode, task.py:117-124), and ``MIPIPE_LOCAL_GPUS`` is the
  number of GPUs of this replica (what task.py counts as ``ngpus_per_node``).  A replica of the
  reference topology (3 replicas x 2 GPUs on one node) therefore owns GPUs [2r, 2r+2) without
  hiding the other four.
* a replica with no accelerators runs on the CPU (``MIPIPE_FORCE_CPU=1``, no visible GPU).
"""
from __future__ import annotations

import os
from typing import Dict, Mapping, Optional

__all__ = ["rank_env", "device_offset", "local_gpus"]


def device_offset(env: Optional[Mapping[str, str]] = None) -> int:
    env = os.environ if env is None else env
    return int(env.get("MIPIPE_DEVICE_OFFSET", "0") or 0)


def local_gpus(env: Optional[Mapping[str, str]] = None) -> Optional[int]:
    """GPUs of this replica (``MIPIPE_LOCAL_GPUS``), or None when the launcher did not say."""
    env = os.environ if env is None else env
    v = env.get("MIPIPE_LOCAL_GPUS")
    return int(v) if v not in (None, "") else None


def rank_env(base: Mapping[str, str], *, master_addr: str, master_port: int,
             world: Optional[int] = None, rank: Optional[int] = None,
             local_rank: Optional[int] = None, local_world: Optional[int] = None,
             group_rank: Optional[int] = None, gpu_offset: int = 0,
             replica_gpus: Optional[int] = None, extra: Optional[Mapping[str, str]] = None,
             rccl: bool = True) -> Dict[str, str]:
    """Environment of one launched process.  ``replica_gpus``: GPUs owned by this process's
    replica (None: leave the GPU variables alone; 0: CPU-only replica)."""
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
            e["MIPIPE_DEVICE_OFFSET"] = str(gpu_offset)
            e["MIPIPE_LOCAL_GPUS"] = str(replica_gpus)
    return e
