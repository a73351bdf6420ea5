"""Spawn one fresh process per local GPU rank (the torchrun contract) from a parent that has
not touched HIP.

The reference's ``mp.spawn(main_worker, nprocs=ngpus_per_node, ...)`` (task.py:117-124) forks
one worker per GPU before any CUDA call.  On MI355X the same rule is stricter: a process that
has initialised the GPU must never fork or exec another GPU program, so the parent here only
builds environments and starts ``N`` brand-new interpreters with ``subprocess`` — it never
imports a HIP-initialising API.  Each child gets ``RANK = LOCAL_RANK = i``,
``WORLD_SIZE = LOCAL_WORLD_SIZE = N``, ``MASTER_ADDR = 127.0.0.1`` and a free
``MASTER_PORT``; all GPUs stay visible to every rank (RCCL needs the peers for xGMI P2P), the
rank selects ``cuda:LOCAL_RANK`` itself — the policy of :mod:`mipipe.launch.env`, whose
:func:`~mipipe.launch.env.rank_env` builds these environments for every launcher.

Output: rank 0's stdout passes through unchanged (``bench.py`` prints its JSON line there);
the other ranks' stdout is redirected to the parent's stderr so the driver still sees exactly
one result line.  Fail-fast: the first rank exiting non-zero terminates the others (SIGTERM,
then SIGKILL after ``grace`` seconds) and its exit code is returned.
"""
from __future__ import annotations

import os
import signal
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence

from .env import rank_env
from .launcher import free_port

__all__ = ["spawn_local_ranks", "rank_envs"]


def rank_envs(nprocs: int, port: Optional[int] = None,
              extra: Optional[Dict[str, str]] = None) -> List[Dict[str, str]]:
    port = port or free_port()
    return [rank_env(os.environ, master_addr="127.0.0.1", master_port=port, world=nprocs,
                     rank=r, local_rank=r, local_world=nprocs, group_rank=0, extra=extra)
            for r in range(nprocs)]


def _terminate(procs: Sequence[subprocess.Popen], grace: float) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except (ProcessLookupError, PermissionError):
                pass
    deadline = time.time() + grace
    for p in procs:
        while p.poll() is None and time.time() < deadline:
            time.sleep(0.05)
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except (ProcessLookupError, PermissionError):
                pass
            p.wait()


def spawn_local_ranks(cmd: Sequence[str], nprocs: int, extra_env: Optional[Dict[str, str]] = None,
                      timeout: Optional[float] = None, grace: float = 10.0) -> int:
    """Run ``cmd`` as ``nprocs`` ranks; return 0, the first failing rank's code, or 124."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    procs: List[subprocess.Popen] = []
    for e in rank_envs(nprocs, extra=extra_env):
        out = None if e["RANK"] == "0" else sys.stderr
        procs.append(subprocess.Popen(list(cmd), env=e, stdout=out, start_new_session=True))
    t0 = time.time()
    rc = 0
    try:
        while True:
            alive = 0
            for p in procs:
                c = p.poll()
                if c is None:
                    alive += 1
                elif c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
            if rc != 0 or alive == 0:
                break
            if timeout is not None and time.time() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    except KeyboardInterrupt:  # pragma: no cover - interactive
        rc = 130
    finally:
        _terminate(procs, grace)
    return rc
