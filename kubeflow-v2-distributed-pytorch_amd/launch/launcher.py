"""Multi-replica / multi-rank process launcher for one MI355X node.

Replaces what Vertex AI Training does for ``CustomTrainingJob.run(replica_count=3,
accelerator_count=2, ...)`` (pytorch-pipeline.ipynb nb:181-188): start the user script on
every replica with the rendezvous env contract task.py consumes — ``WORLD_SIZE``
(replicas), ``RANK`` (replica index), ``MASTER_ADDR``, ``MASTER_PORT``, ``AIP_MODEL_DIR``
(task.py:61, 80, 98, 141, 289) — and, in ``nproc_per_node`` mode, the torchrun contract
(``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``LOCAL_WORLD_SIZE`` per GPU rank).

MI355X specifics: each replica OWNS a disjoint slice of the node's GPUs (one process per GPU is
the RCCL/xGMI sweet spot).  ``gpu_visibility`` picks how the slice is presented
(:mod:`mipipe.launch.env`): ``"slice"`` narrows ``HIP_VISIBLE_DEVICES`` to the replica's GPUs
(what a Vertex VM looks like: the unmodified reference task.py, which counts
``torch.cuda.device_count()`` GPUs (task.py:102), stays on its slice); ``"all"`` keeps every GPU
visible and names the slice by ``MIPIPE_DEVICE_OFFSET`` / ``MIPIPE_LOCAL_GPUS`` (RCCL's xGMI
P2P/IPC transport needs the peers visible — opt-in for mipipe-aware programs).  ``"auto"``
(default) is "slice" unless one replica owns every GPU, or ``MIPIPE_GPU_VISIBILITY`` says
otherwise.  ``HSA_ENABLE_IPC_MODE_LEGACY=0`` is forced so RCCL's dmabuf IPC works.

Failure semantics: fail-fast — the first replica that exits non-zero causes
every other replica's process group to get SIGTERM, then SIGKILL after a grace period; the
launcher returns that first non-zero exit code.  An optional wall-clock ``timeout`` turns a
hang into a failure (exit code 124).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

from .env import rank_env

__all__ = ["LaunchSpec", "launch", "free_port", "visible_gpu_ids", "visible_gpu_source",
           "ReplicaResult"]


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpu_source(env=None):
    """``(variable, ids)``: the GPU ids this launcher may hand out and the variable they came
    from (None: no outer mask, ids are the node's device indices).  HIP numbers devices relative
    to the ROCR-filtered set, so a slice must be written back into the SAME variable: ids read
    from ``ROCR_VISIBLE_DEVICES`` (e.g. under Slurm) are physical and only mean something to
    ROCR, ids read from ``HIP/CUDA_VISIBLE_DEVICES`` are relative to whatever ROCR exposes."""
    env = os.environ if env is None else env
    for var in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None and v.strip() != "":
            return var, [x.strip() for x in v.split(",") if x.strip() != ""]
    n = _count_gpus()
    return None, [str(i) for i in range(n)]


def visible_gpu_ids() -> List[str]:
    """GPU ids this launcher may hand out (honours an outer HIP/CUDA/ROCR_VISIBLE_DEVICES)."""
    return visible_gpu_source()[1]


def _count_gpus() -> int:
    n = os.environ.get("MIPIPE_NUM_GPUS")
    if n is not None:
        return int(n)
    # Count render nodes of AMD GPUs without initialising HIP in this process.
    try:
        import glob
        cnt = 0
        for d in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            with open(d) as f:
                props = f.read()
            if "simd_count" in props and "simd_count 0" not in props:
                cnt += 1
        return cnt
    except Exception:
        return 0


@dataclass
class LaunchSpec:
    command: List[str]                      # e.g. [sys.executable, "task.py", "--dist-url=env://"]
    replica_count: int = 1
    accelerator_count: int = 0              # GPUs per replica
    nproc_per_node: Optional[int] = None    # None: one process per replica (Vertex mode)
    env: Dict[str, str] = field(default_factory=dict)
    model_dir: Optional[str] = None         # AIP_MODEL_DIR
    checkpoint_dir: Optional[str] = None
    tensorboard_dir: Optional[str] = None
    master_addr: str = "127.0.0.1"
    master_port: Optional[int] = None
    log_dir: Optional[str] = None
    echo: bool = True
    timeout: Optional[float] = None
    grace_period: float = 10.0
    cwd: Optional[str] = None
    gpu_visibility: str = "auto"            # "auto" | "slice" | "all" (see module docstring)


@dataclass
class ReplicaResult:
    rank: int
    returncode: Optional[int]
    log_path: Optional[str]


def _pump(proc: subprocess.Popen, prefix: str, log_path: Optional[str], echo: bool) -> None:
    logf = open(log_path, "a") if log_path else None
    try:
        for line in proc.stdout:
            if logf:
                logf.write(line)
                logf.flush()
            if echo:
                sys.stdout.write(f"{prefix}{line}")
                sys.stdout.flush()
    finally:
        if logf:
            logf.close()


def _kill_group(p: subprocess.Popen, sig) -> None:
    try:
        os.killpg(p.pid, sig)
    except (ProcessLookupError, PermissionError):
        pass


def build_envs(spec: LaunchSpec) -> List[Dict[str, str]]:
    """Environment of every process the launch starts (exposed for tests)."""
    src_var, gpus = visible_gpu_source()
    # a slice is written back into the variable the ids came from (ROCR ids are physical)
    slice_var = "ROCR_VISIBLE_DEVICES" if src_var == "ROCR_VISIBLE_DEVICES" else "HIP_VISIBLE_DEVICES"
    per_replica = spec.accelerator_count
    nproc = spec.nproc_per_node
    total_needed = spec.replica_count * per_replica
    if per_replica and total_needed > len(gpus):
        raise RuntimeError(f"job needs {spec.replica_count}x{per_replica}={total_needed} GPUs, "
                           f"node exposes {len(gpus)} ({gpus})")
    mode = spec.gpu_visibility
    if mode == "auto":
        mode = os.environ.get("MIPIPE_GPU_VISIBILITY", "auto")
    if mode == "auto":
        mode = "all" if (not per_replica or total_needed == len(gpus)) else "slice"
    if mode not in ("slice", "all"):
        raise ValueError(f"gpu_visibility must be auto, slice or all, not {mode!r}")
    port = spec.master_port or free_port()
    envs = []
    procs_per_replica = nproc or 1
    world = spec.replica_count * procs_per_replica
    for r in range(spec.replica_count):
        for lr in range(procs_per_replica):
            if nproc:
                if per_replica and lr >= per_replica:
                    raise RuntimeError(f"nproc_per_node={nproc} exceeds accelerator_count={per_replica}")
                ids = dict(world=world, rank=r * procs_per_replica + lr, local_rank=lr,
                           local_world=procs_per_replica, group_rank=r)
            else:  # one process per replica that spawns its GPU workers (task.py:117-124)
                ids = dict(world=spec.replica_count, rank=r)
            own = gpus[r * per_replica:(r + 1) * per_replica]
            e = rank_env(os.environ, master_addr=spec.master_addr, master_port=port,
                         gpu_offset=r * per_replica, replica_gpus=per_replica, extra=spec.env,
                         visible=",".join(own) if (mode == "slice" and per_replica) else None,
                         visible_var=slice_var, **ids)
            if spec.model_dir:
                e["AIP_MODEL_DIR"] = spec.model_dir
            if spec.checkpoint_dir:
                e["AIP_CHECKPOINT_DIR"] = spec.checkpoint_dir
            if spec.tensorboard_dir:
                e["AIP_TENSORBOARD_LOG_DIR"] = spec.tensorboard_dir
            e["CLUSTER_SPEC"] = (
                '{"cluster": {"workerpool0": ["%s:%d"]}, "task": {"type": "workerpool0", "index": %d}}'
                % (spec.master_addr, port, r))
            envs.append(e)
    return envs


def launch(spec: LaunchSpec) -> int:
    """Run the job; return 0 or the first failing process' exit code (124 on timeout).

    Uses the native supervisor (csrc/runtime/supervisor.cpp) when built, else a
    subprocess-based equivalent with the same semantics."""
    from mipipe.runtime import runtime, runtime_available
    if runtime_available():
        return _launch_native(spec, runtime())
    return _launch_python(spec)


def _launch_native(spec: LaunchSpec, rt) -> int:
    envs = build_envs(spec)
    if spec.log_dir:
        os.makedirs(spec.log_dir, exist_ok=True)
    pg = rt.ProcessGroup(echo=spec.echo)
    for i, e in enumerate(envs):
        log_path = os.path.join(spec.log_dir, f"rank{i}.log") if spec.log_dir else ""
        pg.spawn(list(spec.command), [f"{k}={v}" for k, v in e.items()], spec.cwd or "",
                 log_path, f"[rank{i}] ")
    try:
        rc = pg.wait(float(spec.timeout or 0.0), float(spec.grace_period))
    except KeyboardInterrupt:  # pragma: no cover - interactive
        pg.interrupt()
        rc = pg.wait(0.0, float(spec.grace_period))
    return int(rc)


def _launch_python(spec: LaunchSpec) -> int:
    envs = build_envs(spec)
    if spec.log_dir:
        os.makedirs(spec.log_dir, exist_ok=True)
    procs: List[subprocess.Popen] = []
    pumps: List[threading.Thread] = []
    for i, e in enumerate(envs):
        log_path = os.path.join(spec.log_dir, f"rank{i}.log") if spec.log_dir else None
        p = subprocess.Popen(spec.command, env=e, cwd=spec.cwd, stdout=subprocess.PIPE,
                             stderr=subprocess.STDOUT, text=True, bufsize=1,
                             start_new_session=True)
        procs.append(p)
        th = threading.Thread(target=_pump, args=(p, f"[rank{i}] ", log_path, spec.echo),
                              daemon=True)
        th.start()
        pumps.append(th)
    t0 = time.time()
    first_fail: Optional[int] = None
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad and first_fail is None:
                first_fail = bad[0]
                break
            if all(c is not None for c in codes):
                break
            if spec.timeout is not None and time.time() - t0 > spec.timeout:
                first_fail = 124
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        first_fail = 130
    if first_fail is not None:
        for p in procs:
            if p.poll() is None:
                _kill_group(p, signal.SIGTERM)
        deadline = time.time() + spec.grace_period
        while time.time() < deadline and any(p.poll() is None for p in procs):
            time.sleep(0.05)
        for p in procs:
            if p.poll() is None:
                _kill_group(p, signal.SIGKILL)
        for p in procs:
            p.wait()
    for th in pumps:
        th.join(timeout=5)
    return 0 if first_fail is None else int(first_fail)
