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

# Channel profiles for the 8-GPU xGMI mesh (``MIPIPE_RCCL_PROFILE``; the environment still wins).
# One RCCL channel is one workgroup on one CU, moving its slice over one ring / tree edge, so the
# channel count trades link parallelism against CUs taken from the kernels it overlaps:
#  * "auto" (default): RCCL's own topology search — it reads the xGMI full mesh (7 links per
#    MI355X) and picks rings and channel counts per message size.  DDP buckets overlap backward
#    here (94.5 % concurrent, profiles/r3_ddp_rccl_overlap_eager_highprio.txt), so the CUs a
#    bigger channel count would take cost more than the link time they would save.
#  * "overlap": at most 8 channels — for steps whose collectives are fully hidden under compute:
#    RCCL takes <= 8 of the 256 CUs from the overlapped kernels.
#  * "bandwidth": at least 32 channels — for exposed collectives (parameter broadcast at start,
#    gradient tails of compute-light models): every xGMI link carries several rings' slices.
RCCL_PROFILES = {
    "auto": {},
    "overlap": {"NCCL_MAX_NCHANNELS": "8"},
    "bandwidth": {"NCCL_MIN_NCHANNELS": "32"},
}


def rccl_profile_env(profile: Optional[str] = None) -> dict:
    """The RCCL variables of ``profile`` (default: ``$MIPIPE_RCCL_PROFILE`` or "auto")."""
    name = profile if profile is not None else os.environ.get("MIPIPE_RCCL_PROFILE", "auto")
    if name not in RCCL_PROFILES:
        raise ValueError(f"MIPIPE_RCCL_PROFILE={name!r}: expected one of {sorted(RCCL_PROFILES)}")
    return dict(RCCL_PROFILES[name])


def configure_rccl_env(env: Optional[dict] = None, profile: Optional[str] = None) -> dict:
    """Apply :data:`RCCL_ENV_DEFAULTS` and the channel profile to ``env`` (``os.environ`` by
    default) without overriding values already set; returns the target mapping.  Must run before
    the first process group / communicator exists (RCCL reads its variables at comm init)."""
    target = os.environ if env is None else env
    prof = rccl_profile_env(profile if profile is not None else target.get("MIPIPE_RCCL_PROFILE"))
    for k, v in list(RCCL_ENV_DEFAULTS.items()) + list(prof.items()):
        target.setdefault(k, v)
    return target


def enable_rccl_transport_log(env: Optional[dict] = None) -> Optional[str]:
    """Send RCCL's INFO log of communicator setup (not per-collective lines) to a per-process file
    so :func:`rccl_transports` can report which transport each peer pair got — the evidence that
    an 8-GPU run used xGMI P2P rather than host shared memory.  Must run before the first
    communicator exists.  Returns the log path, or None when the caller already routes NCCL_DEBUG
    elsewhere (or ``MIPIPE_RCCL_TRANSPORT_LOG=0``)."""
    import tempfile
    target = os.environ if env is None else env
    if target.get("MIPIPE_RCCL_TRANSPORT_LOG", "1") == "0":
        return None
    if "NCCL_DEBUG" in target and "NCCL_DEBUG_FILE" not in target:
        return None
    d = target.get("MIPIPE_RCCL_LOG_DIR") or tempfile.gettempdir()
    target.setdefault("NCCL_DEBUG", "INFO")
    target.setdefault("NCCL_DEBUG_SUBSYS", "INIT,P2P,SHM,NET,GRAPH")
    target.setdefault("NCCL_DEBUG_FILE", os.path.join(d, f"mipipe_rccl.{os.getpid()}.log"))
    return target["NCCL_DEBUG_FILE"]


_VIA = None


def rccl_transports(path: Optional[str]) -> Optional[dict]:
    """Parse RCCL channel-setup lines (``Channel 00/0 : 0[0] -> 1[1] via P2P/IPC``) from an INFO
    log: ``{"transports": {"P2P/IPC": n, ...}, "pairs": {"0->1": "P2P/IPC", ...}}``, or None
    when the log is missing or has no such lines."""
    global _VIA
    import re
    if not path or not os.path.exists(path):
        return None
    if _VIA is None:
        _VIA = re.compile(r"(\d+)\[[^\]]*\]\s*->\s*(\d+)\[[^\]]*\].*?\bvia\s+([A-Za-z0-9_]+(?:/[A-Za-z0-9_]+)?)")
    counts: dict = {}
    pairs: dict = {}
    with open(path, errors="replace") as f:
        for line in f:
            m = _VIA.search(line)
            if not m:
                continue
            t = m.group(3)
            counts[t] = counts.get(t, 0) + 1
            pairs.setdefault(f"{m.group(1)}->{m.group(2)}", t)
    if not counts:
        return None
    return {"transports": counts, "pairs": dict(sorted(pairs.items()))}


def rccl_settings(env: Optional[dict] = None) -> dict:
    """The RCCL / ProcessGroupNCCL variables in effect (recorded with every bench line)."""
    src = os.environ if env is None else env
    keys = sorted(k for k in src if k.startswith(("NCCL_", "RCCL_", "TORCH_NCCL_")) or
                  k == "MIPIPE_RCCL_PROFILE")
    return {k: src[k] for k in keys}


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
