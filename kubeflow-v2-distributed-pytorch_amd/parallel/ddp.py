"""DistributedDataParallel over RCCL with flat in-place gradient buckets.

Replaces ``torch.nn.parallel.DistributedDataParallel(model, device_ids=[gpu])`` used by the
reference (task.py:189, 194) and reproduces its collective contract:

* C2 — at construction, all ranks agree on parameter shapes (all-gather of a digest);
* C3 — at construction, parameters and buffers are broadcast from rank 0 (the flat
  parameter buffer goes in ONE collective);
* C4 — before every grad-enabled forward, module buffers (BN running stats) are broadcast
  from rank 0 (``broadcast_buffers=True``, DDP's default);
* C5 — during backward, gradients are averaged with bucketed all-reduce overlapped with the
  remaining backward kernels.

MI355X design: gradients already live in one flat fp32 buffer in gradient-ready order
(:mod:`mipipe.optim.flat`), so a bucket is a contiguous slice that RCCL all-reduces *in place*
— no copy into/out of bucket staging buffers.  Buckets are launched strictly in index order
(every rank issues the same collective sequence) from post-accumulate-grad hooks, on the
process group's communication stream; the step's end waits on them with stream semantics only
(no host sync).  Bucket size defaults to 32 MiB (≈7 links × ~4.5 MiB chunks per ring step on
the 8-GPU xGMI mesh) with a small first bucket so communication starts early and a small last
bucket so little is left to all-reduce after the final backward kernel; the optional
``comm_dtype=torch.bfloat16`` halves the bytes on the wire.

Reducer: the native C++ reducer (``mipipe._C.Reducer``, csrc/comm/reducer.cpp) counts bucket
readiness from post hooks on the AccumulateGrad nodes and from the HIP kernels that write
gradients straight into the flat buffer, launches each bucket's all-reduce through the c10d
process group, and makes the compute stream wait on them at the end of backward — no Python
frame per parameter.  With ``comm_dtype=torch.bfloat16`` one HIP pass packs a bucket into a bf16
wire buffer pre-scaled by 1/world and one pass widens the reduced bucket back.  The pure-Python
reducer below is the fallback when ``_C`` is not built (``MIPIPE_NATIVE_REDUCER=0`` forces it);
both issue the identical collective sequence.

Tied embeddings (BERT's MLM decoder shares the word-embedding weight, SURVEY §2.6 C5''): the
weight's gradient has a dense part (the decoder's weight-grad, done at the START of the backward)
and a sparse part (the lookup's scatter of one row per token, the LAST backward op).  A plain
bucketed all-reduce of the 94 MB weight could only start after the scatter — fully exposed.
Here (``sparse_embedding=True``, the default; ``MIPIPE_SPARSE_EMBEDDING=0`` turns it off) the
weight's flat slot goes first, the dense part is all-reduced in the first bucket while the
encoder's backward runs, and the lookup part travels as (token id, row) pairs: one
``all_gather`` of the ids and one of the rows (bf16 on the GPU: 6.3 MB per rank at 32 x 128),
issued after the last bucket, then every rank scatters every rank's rows, times 1/world, in rank
order through the ordered embedding backward (one writer per table row, stable id order) — the
same sum on every rank, bit for bit.

Debug aid (SURVEY §5.2 hazard): ``check_collectives=True`` (or ``MIPIPE_CHECK_COLLECTIVES=1``)
hashes every collective this wrapper issues and compares the digests across ranks every
``check_every`` steps, turning a mismatched collective sequence into an immediate error.
"""
from __future__ import annotations

import contextlib
import hashlib
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as tnn

from mipipe.optim.flat import FlatParamSpace, get_flat_space

__all__ = ["DistributedDataParallel", "CollectiveSequenceError", "Bucket"]


_DEBUG = os.environ.get("MIPIPE_DDP_DEBUG", "0") == "1"


class CollectiveSequenceError(RuntimeError):
    pass


class Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "work", "launched", "tmp")

    def __init__(self, index: int, start: int, end: int, params: List[tnn.Parameter]):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.pending = len(params)
        self.work = None
        self.launched = False
        self.tmp = None

    @property
    def nbytes(self) -> int:
        return (self.end - self.start) * 4


class _CollectiveLog:
    def __init__(self):
        self.h = hashlib.sha1()
        self.count = 0

    def record(self, op: str, t: torch.Tensor) -> None:
        self.record_shape(op, t.numel(), t.dtype)

    def record_shape(self, op: str, numel: int, dtype) -> None:
        self.h.update(f"{op}:{numel}:{dtype};".encode())
        self.count += 1

    def digest(self) -> bytes:
        return self.h.digest()


class _SparseRowExchange:
    """The lookup part of a tied embedding weight's gradient, exchanged as (id, row) pairs.

    Installed as ``param._mipipe_sparse_sink``.  The ids are known at FORWARD time, so the
    embedding op hands them over there (:meth:`on_forward`): their ``all_gather`` is issued at
    once, and the stable sort of the world's ids that the ordered scatter needs runs on a side
    stream during the forward (:meth:`after_forward`) — after the last backward kernel only the
    rows' ``all_gather`` and the scatter are left.  The backward hands over the per-token
    gradient rows instead of scattering them (ops/functional.py ``_EmbeddingFn``).

    Fixed-capacity protocol: ``all_gather_into_tensor`` needs equal sizes on every rank, so the
    capacity is agreed once (the largest first-step token count, one host exchange) and every
    later step pads its ids with -1 (skipped by the scatter) and its rows with zeros up to it.
    A ragged / dynamically padded batch with fewer tokens therefore still matches; a step with
    MORE tokens than the capacity raises on the rank that grew, before that rank issues any
    collective.  Its peers have no way to know without a host round trip per step (which a
    captured hipGraph step cannot make), so they block in the ids ``all_gather`` until the job
    is torn down: mipipe's launchers are fail-fast (the raising rank's non-zero exit SIGTERMs
    every other rank, launch/launcher.py), and otherwise the process group's timeout or the
    transport's peer-closed error ends them — never a silently mismatched collective
    (``tests/test_optim_ddp.py::test_ddp_sparse_capacity_one_rank_grows``).  The capacity is
    part of the collective digest (``check_collectives``)."""

    def __init__(self, ddp: "DistributedDataParallel", param: tnn.Parameter):
        self.ddp = ddp
        self.param = param
        self.pending = None
        self.cap: Optional[int] = None
        self.fwd = None          # {n, ids_all, work, sorted, event} of the current step
        self.sent_bytes = 0      # per rank, last exchange (ids + rows)
        self.ids_issued_in_forward = 0  # steps whose ids gather was issued by the forward

    def _active(self) -> bool:
        return self.ddp._comm and self.ddp._sync_enabled

    def _capacity(self, n: int) -> int:
        if self.cap is None:
            ns: List[Optional[int]] = [None] * self.ddp.world
            dist.all_gather_object(ns, int(n), group=self.ddp.process_group)
            self.cap = max(int(v) for v in ns)
        if n > self.cap:
            raise RuntimeError(
                f"DDP sparse embedding exchange: {n} tokens this step exceed the capacity of "
                f"{self.cap} agreed at the first step (all ranks' maximum); build the DDP wrapper "
                "on the largest batch shape or pass sparse_embedding=False")
        return self.cap

    def on_forward(self, idx: torch.Tensor) -> None:
        """Grad-enabled forward of the lookup: issue the ids' all_gather now."""
        if not self._active():
            self.fwd = None
            return
        idx = idx.reshape(-1)
        n = int(idx.numel())
        cap = self._capacity(n)
        ids = idx if n == cap else torch.cat([idx, idx.new_full((cap - n,), -1)])
        ddp = self.ddp
        ids_all = ids.new_empty(ddp.world * cap)
        ddp._clog.record("all_gather", ids)
        work = dist.all_gather_into_tensor(ids_all, ids.contiguous(), group=ddp.process_group,
                                           async_op=True)
        self.fwd = {"n": n, "ids_all": ids_all, "work": work, "sorted": None, "event": None}
        self.ids_issued_in_forward += 1

    def after_forward(self) -> None:
        """Stable-sort the gathered ids (rank order, then position: the scatter's summation
        order) on a side stream that waits for the gather — off the compute stream's path."""
        f = self.fwd
        if f is None or f["sorted"] is not None:
            return
        ids_all = f["ids_all"]
        if not ids_all.is_cuda:
            f["work"].wait()
            f["sorted"] = torch.sort(ids_all, stable=True)
            return
        from mipipe.ops.functional import _side_stream
        cur = torch.cuda.current_stream(ids_all.device)
        side = _side_stream(ids_all)
        side.wait_stream(cur)  # fork from the compute stream (joins a hipGraph capture too)
        with torch.cuda.stream(side):
            f["work"].wait()  # stream semantics: the side stream waits for the gather
            sid, perm = torch.sort(ids_all, stable=True)
        for t in (sid, perm):
            t.record_stream(cur)
        ev = torch.cuda.Event()
        ev.record(side)
        f["sorted"], f["event"] = (sid, perm), ev

    def __call__(self, idx: torch.Tensor, dy: torch.Tensor) -> None:
        idx = idx.reshape(-1)
        dy = dy.reshape(-1, dy.shape[-1])
        if not self._active():  # no_sync(): a local scatter, like no DDP
            self._scatter(dy, idx, 1.0)
            return
        if self.fwd is None or self.fwd["n"] != idx.numel():
            self.on_forward(idx)  # forward ran outside this wrapper: gather the ids now
        self.after_forward()
        self.pending = dy
        # after the reducer's end-of-backward callback (queued at the first ready gradient):
        # every bucket, the dense part of this weight included, is reduced by then
        torch.autograd.Variable._execution_engine.queue_callback(self._exchange)

    def _scatter(self, rows, ids, scale, presorted=None):
        from mipipe.ops import kernels as K
        from mipipe.optim.flat import flat_space_for
        fs = flat_space_for(self.param)
        K.embedding_bwd(rows.contiguous(), ids.contiguous(), self.param.shape[0],
                        fs.grad_view(self.param), ordered=True, scale=scale, presorted=presorted)

    def _exchange(self) -> None:
        dy, f = self.pending, self.fwd
        self.pending, self.fwd = None, None
        ddp = self.ddp
        world, pg = ddp.world, ddp.process_group
        n, H = dy.shape
        cap = self.cap
        if n < cap:
            dy = torch.cat([dy, dy.new_zeros(cap - n, H)])
        rows_all = dy.new_empty(world * cap, H)
        ddp._clog.record("all_gather", dy)
        w = dist.all_gather_into_tensor(rows_all, dy.contiguous(), group=pg, async_op=True)
        w.wait()  # stream semantics on RCCL: the compute stream waits, the host does not
        if f["event"] is not None:
            torch.cuda.current_stream(dy.device).wait_event(f["event"])
        self.sent_bytes = cap * (8 + H * dy.element_size())
        # rank order is the all_gather order; the ordered scatter sums equal ids in that order
        self._scatter(rows_all, f["ids_all"], 1.0 / world, presorted=f["sorted"])


class DistributedDataParallel(tnn.Module):
    def __init__(self, module: tnn.Module, device_ids: Optional[List[int]] = None,
                 output_device=None, broadcast_buffers: bool = True,
                 process_group=None, bucket_cap_mb: float = 32.0, first_bucket_mb: float = 1.0,
                 last_bucket_mb: float = 2.0,
                 comm_dtype: Optional[torch.dtype] = None, find_unused_parameters: bool = False,
                 check_collectives: Optional[bool] = None, check_every: int = 50,
                 gradient_as_bucket_view: bool = True, static_graph: bool = False,
                 force_reduce: Optional[bool] = None, sparse_embedding: Optional[bool] = None):
        super().__init__()
        self.module = module
        self.device_ids = device_ids
        self.broadcast_buffers = broadcast_buffers
        self.process_group = process_group
        self.comm_dtype = comm_dtype
        self.require_forward_param_sync = True
        self._sync_enabled = True
        if check_collectives is None:
            check_collectives = os.environ.get("MIPIPE_CHECK_COLLECTIVES", "0") == "1"
        self.check_collectives = check_collectives
        self.check_every = check_every
        self._clog = _CollectiveLog()
        self._steps = 0
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        # force_reduce (or MIPIPE_DDP_FORCE_REDUCE=1): issue every collective even at world
        # size 1, so the RCCL path (buffer broadcast, bucket all-reduces, their overlap with
        # backward and their capture into a hipGraph) runs and can be profiled on one GPU.
        if force_reduce is None:
            force_reduce = os.environ.get("MIPIPE_DDP_FORCE_REDUCE", "0") == "1"
        self.force_reduce = bool(force_reduce) and dist.is_initialized()
        self._comm = self.world > 1 or self.force_reduce
        params = [p for p in module.parameters() if p.requires_grad]
        dev = params[0].device
        # compute-dtype weight shadow: bf16 on the GPU unless the model computes in fp32 (the
        # reference's precision), whose kernels read the fp32 master weights directly
        cdt = getattr(module, "compute_dtype", None)
        shadow = torch.bfloat16 if dev.type == "cuda" and cdt != torch.float32 else None
        if sparse_embedding is None:
            sparse_embedding = os.environ.get("MIPIPE_SPARSE_EMBEDDING", "1") == "1"
        tied = [p for p in params if getattr(p, "_mipipe_tied_later", False)]
        want_sparse = bool(sparse_embedding) and self._comm and bool(tied)
        if want_sparse:
            from mipipe.optim.flat import flat_space_for
            if any(flat_space_for(p) is not None for p in params):
                want_sparse = False  # the flat order is fixed already (optimizer built first)
            else:
                for p in tied:
                    p._mipipe_flat_first = True  # ready at the start of the backward
        self.space: FlatParamSpace = get_flat_space(params, shadow, module)
        self._sparse: List[_SparseRowExchange] = []
        if want_sparse:
            for p in tied:
                ex = _SparseRowExchange(self, p)
                p._mipipe_sparse_sink = ex
                self._sparse.append(ex)
        backend = dist.get_backend(process_group) if dist.is_initialized() else "none"
        self._avg_supported = backend == "nccl"
        # latency path for the per-forward buffer broadcast (C4): one-shot over IPC peer
        # pointers (parallel/oneshot.py) when MIPIPE_ONESHOT=1 on a single-node GPU job
        self._oneshot = None
        if self._comm and dev.type == "cuda":
            from mipipe.parallel.oneshot import OneShotComm, oneshot_enabled
            if oneshot_enabled():
                self._oneshot = OneShotComm(process_group, device=dev)
        if self._comm:
            self._verify_shapes(params)
            self._sync_module_states()
        self.buckets = self._build_buckets(bucket_cap_mb * 2 ** 20, first_bucket_mb * 2 ** 20,
                                           last_bucket_mb * 2 ** 20)
        self._bucket_of = {}
        for b in self.buckets:
            for p in b.params:
                self._bucket_of[id(p)] = b
        self._next_bucket = 0
        self._callback_queued = False
        self._reported = set()
        self._reducer = self._make_native_reducer() if self._comm else None
        if self._reducer is not None:
            self._slot_of = {id(p): i for i, (_, _, p) in enumerate(self.space.ranges())}
            self._reducer.register_hooks([r[2] for r in self.space.ranges()])
            self._hooks = []
            # kernels that write weight gradients straight into the flat buffer report here
            self.space.add_ready_listener(self._native_ready)
        else:
            self._hooks = [p.register_post_accumulate_grad_hook(self._on_ready) for p in params]
            self.space.add_ready_listener(self._on_ready)

    def _make_native_reducer(self):
        if os.environ.get("MIPIPE_NATIVE_REDUCER", "1") == "0":
            return None
        from mipipe.ops._native import native, native_available
        if not native_available():
            return None
        if self.comm_dtype not in (None, torch.float32, torch.bfloat16):
            return None
        pg = self.process_group if self.process_group is not None else dist.group.WORLD
        slot_bucket = []
        for b in self.buckets:
            slot_bucket += [b.index] * len(b.params)
        return native().Reducer(pg.group_name, self.space.flat_grad,
                                [(b.start, b.end) for b in self.buckets], slot_bucket,
                                self.world, self._avg_supported,
                                self.comm_dtype == torch.bfloat16)

    @property
    def native_reducer(self) -> bool:
        return self._reducer is not None

    def _native_ready(self, param) -> None:
        slot = self._slot_of.get(id(param))
        if slot is not None:
            self._reducer.mark_ready(slot)

    # ------------------------------------------------------------------ construction
    def _verify_shapes(self, params) -> None:
        h = hashlib.sha1(";".join(f"{tuple(p.shape)}:{p.dtype}" for p in params).encode()).hexdigest()
        out: List[Optional[str]] = [None] * self.world
        dist.all_gather_object(out, h, group=self.process_group)
        if any(o != h for o in out):
            raise RuntimeError(f"DDP: parameter shapes differ across ranks: {out}")

    def _broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        self._clog.record("broadcast", t)
        dist.broadcast(t, src, group=self.process_group)

    def _sync_module_states(self) -> None:
        self._broadcast(self.space.flat)
        self.space.sync_shadow()
        self._broadcast_buffers_now()

    def _module_buffers(self) -> List[torch.Tensor]:
        return [b for b in self.module.buffers()]

    def _flatten_buffers(self) -> None:
        """Re-home every module buffer as a view of one flat tensor per dtype, so the per-step
        buffer broadcast (C4) is a single in-place collective per dtype instead of a cat, a
        broadcast and one copy kernel per buffer (~160 tiny kernels for ResNet-50)."""
        self._flat_bufs = []
        by_dtype = {}
        for mod in self.module.modules():
            for name, b in mod._buffers.items():
                if b is not None:
                    by_dtype.setdefault(b.dtype, []).append((mod, name, b))
        for dt, lst in by_dtype.items():
            parts = [b.detach().reshape(-1) for _, _, b in lst]
            esz = parts[0].element_size()
            pad = (-sum(p.numel() for p in parts) * esz) % 16 // esz  # 16-B multiple (one-shot)
            if pad:
                parts.append(torch.zeros(pad, dtype=dt, device=parts[0].device))
            flat = torch.cat(parts)
            off = 0
            for mod, name, b in lst:
                n = b.numel()
                mod._buffers[name] = flat[off:off + n].view_as(b)
                off += n
            self._flat_bufs.append(flat)

    def _broadcast_buffers_now(self) -> None:
        if getattr(self, "_flat_bufs", None) is None:
            self._flatten_buffers()
        for flat in self._flat_bufs:
            self._broadcast(flat)

    def _broadcast_buffers_async(self) -> None:
        """C4: the per-forward buffer broadcast (BN running stats, ~38 KB for ResNet-18) as one
        collective per dtype on the comm stream; :meth:`_wait_buffer_sync` makes the compute
        stream wait for it (the host does not block on RCCL).  The wait comes before the module
        runs: the fused conv -> BN paths read ``running_mean`` (the statistics shift) and update
        the running statistics in place without calling the BatchNorm module, so no per-module
        hook can place the wait later without racing the broadcast (measured: a hook on the
        buffer owners left the 4-rank gloo run nondeterministic)."""
        if getattr(self, "_flat_bufs", None) is None:
            self._flatten_buffers()
        works = []
        for flat in self._flat_bufs:
            self._clog.record("broadcast", flat)
            if self._oneshot is not None and self._oneshot.fits(flat):
                self._oneshot.broadcast(flat, 0)  # one IPC hop, ordered on the compute stream
            else:
                works.append(dist.broadcast(flat, 0, group=self.process_group, async_op=True))
        self._pending_buffer_work = works

    def _wait_buffer_sync(self, module=None, args=None) -> None:
        works = getattr(self, "_pending_buffer_work", None)
        if works:
            self._pending_buffer_work = None
            for w in works:
                w.wait()  # stream semantics on RCCL: the compute stream waits, the host does not

    def _build_buckets(self, cap_bytes: float, first_bytes: float,
                       last_bytes: float = 0.0) -> List[Bucket]:
        """Contiguous flat-gradient slices in gradient-ready order: a small FIRST bucket (the
        classifier: communication starts as soon as backward does), a small LAST bucket (the
        stem and first layers: the only all-reduce that cannot overlap backward is this one, so
        its bytes are the exposed communication of the step), and the rest split into equal
        buckets of at most ``cap_bytes``.  With a plain greedy cut the tail of ResNet-50 would be
        a ~27 MB remainder (layer 2 + layer 1 + stem) all-reduced after the last kernel."""
        ranges = list(self.space.ranges())
        n = len(ranges)
        cuts = []  # exclusive end index of each bucket
        i, acc = 0, 0
        while i < n:  # first bucket
            acc += (ranges[i][1] - ranges[i][0]) * 4
            i += 1
            if acc >= first_bytes:
                break
        cuts.append(i)
        j, acc = n, 0
        if last_bytes > 0:
            while j > i:  # last bucket, from the end: at most last_bytes (at least one param)
                nb = (ranges[j - 1][1] - ranges[j - 1][0]) * 4
                if acc > 0 and acc + nb > last_bytes:
                    break
                acc += nb
                j -= 1
        if j > i:  # middle: equal buckets of <= cap_bytes
            mid = sum((ranges[k][1] - ranges[k][0]) * 4 for k in range(i, j))
            nb = max(1, int(-(-mid // max(cap_bytes, 1.0))))
            target = mid / nb
            acc = 0
            for k in range(i, j):
                acc += (ranges[k][1] - ranges[k][0]) * 4
                if acc >= target and k + 1 < j:
                    cuts.append(k + 1)
                    acc = 0
            cuts.append(j)
        if cuts[-1] != n:
            cuts.append(n)
        buckets: List[Bucket] = []
        lo = 0
        for hi in cuts:
            if hi <= lo:
                continue
            ps = [r[2] for r in ranges[lo:hi]]
            buckets.append(Bucket(len(buckets), ranges[lo][0], ranges[hi - 1][1], ps))
            lo = hi
        return buckets

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kwargs):
        if self._comm and torch.is_grad_enabled() and self.broadcast_buffers \
                and self.require_forward_param_sync:
            self._broadcast_buffers_async()
            self._wait_buffer_sync()
        if torch.is_grad_enabled() and self.module.training:
            self._prepare_backward()
            self.require_forward_param_sync = True
        else:
            self.require_forward_param_sync = False
        out = self.module(*args, **kwargs)
        for ex in self._sparse:
            ex.after_forward()
        return out

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync_enabled
        self._sync_enabled = False
        if self._reducer is not None:
            self._reducer.prepare(False)
        try:
            yield
        finally:
            self._sync_enabled = old

    # ------------------------------------------------------------------ backward / comm
    def _prepare_backward(self) -> None:
        if self._reducer is not None:
            on = self._comm and self._sync_enabled
            self._reducer.prepare(on)
            self.space.ensure_grad_views()
            if on:
                # the native reducer issues exactly this sequence during the coming backward
                wdt = torch.bfloat16 if self._reducer.wire_bf16 else torch.float32
                for b in self.buckets:
                    self._clog.record_shape("all_reduce", b.end - b.start, wdt)
                self._steps += 1
                if self.check_collectives and self._steps % self.check_every == 0:
                    self._verify_when_safe()
            return
        self._reported = set()
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
            b.launched = False
            b.tmp = None
        self._next_bucket = 0
        self._callback_queued = False
        self.space.ensure_grad_views()

    def _on_ready(self, param) -> None:
        if not self._comm or not self._sync_enabled:
            return
        b = self._bucket_of.get(id(param))
        if b is None:
            return
        # A parameter can be reported twice: by the kernel that wrote its gradient straight into
        # the flat buffer (space listener) AND by autograd's post-accumulate hook, which fires
        # even when the Function returned no gradient for it.  Counting it twice would launch
        # the bucket's all-reduce before its other gradients exist.
        if id(param) in self._reported:
            return
        self._reported.add(id(param))
        if _DEBUG and dist.get_rank() == 0:
            print(f"[ddp r0] ready {tuple(param.shape)} bucket {b.index} "
                  f"max={float(self.space.grad_view(param).abs().max()):.3e}", flush=True)
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        b.pending -= 1
        self._launch_ready()

    def _launch(self, b: Bucket) -> None:
        g = self.space.flat_grad[b.start:b.end]
        if self.comm_dtype is not None and self.comm_dtype != g.dtype:
            b.tmp = g.to(self.comm_dtype)
            t = b.tmp
        else:
            t = g
        self._clog.record("all_reduce", t)
        if _DEBUG:
            print(f"[ddp r{dist.get_rank()}] launch bucket {b.index} [{b.start},{b.end}) "
                  f"params={len(b.params)} norm={float(t.float().norm()):.4e}", flush=True)
        op = dist.ReduceOp.AVG if self._avg_supported else dist.ReduceOp.SUM
        b.work = dist.all_reduce(t, op=op, group=self.process_group, async_op=True)
        b.launched = True

    def _launch_ready(self) -> None:
        while self._next_bucket < len(self.buckets) and self.buckets[self._next_bucket].pending <= 0:
            self._launch(self.buckets[self._next_bucket])
            self._next_bucket += 1

    def _finalize(self) -> None:
        # unused parameters: their (zero) gradients still take part in the average
        while self._next_bucket < len(self.buckets):
            self._launch(self.buckets[self._next_bucket])
            self._next_bucket += 1
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                g = self.space.flat_grad[b.start:b.end]
                if _DEBUG:
                    print(f"[ddp r{dist.get_rank()}] done bucket {b.index} "
                          f"norm={float(g.float().norm()):.4e}", flush=True)
                if b.tmp is not None:
                    g.copy_(b.tmp)
                    if not self._avg_supported:
                        g.div_(self.world)
                elif not self._avg_supported:
                    g.div_(self.world)
                b.work = None
                b.tmp = None
        self._steps += 1
        if self.check_collectives and self._steps % self.check_every == 0:
            self._verify_when_safe()

    # ------------------------------------------------------------------ debugging
    def check_comm_errors(self, final: bool = False) -> None:
        """Raise :class:`CollectiveSequenceError` if a one-shot collective gave up waiting for a
        peer.  Cheap (no host sync) unless ``final``; the trainer calls it at every
        log interval and once at the end.  RCCL collectives fail through the process group's
        own timeout instead."""
        if self._oneshot is not None:
            self._oneshot.check(final=final)

    def _verify_when_safe(self) -> None:
        """The digest exchange synchronises the host with every rank: never inside a hipGraph
        capture (warm-up / capture of a graphed step); that check is skipped, the next one covers it
        (the digest accumulates every collective)."""
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return
        self.verify_collective_sequence()

    def verify_collective_sequence(self) -> None:
        """All-gather the per-rank digest of collectives issued so far; raise on mismatch."""
        d = (self._clog.digest().hex(), self._clog.count)
        out: List[Optional[Tuple[str, int]]] = [None] * self.world
        dist.all_gather_object(out, d, group=self.process_group)
        if any(o != out[0] for o in out):
            raise CollectiveSequenceError(
                f"collective sequences diverged across ranks: {out} (an op ran on a subset of "
                "ranks — e.g. evaluating the DDP wrapper on rank 0 only, SURVEY §5.2)")

    def state_dict(self, *args, **kwargs):
        return super().state_dict(*args, **kwargs)
