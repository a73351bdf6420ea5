"""Fused flat-buffer optimizers vs torch.optim, and DDP over gloo (world size 2)."""
import copy
import os

import pytest
import torch
import torch.multiprocessing as mp

from mipipe.optim import SGD, AdamW, flat_space_for
from mipipe.ops import functional as MF
from mipipe import nn as mnn


class MLP(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.fc1 = mnn.Linear(16, 32)
        self.fc2 = mnn.Linear(32, 8)

    def forward(self, x):
        return self.fc2(self.fc1(x, act="relu"))


def test_sgd_matches_torch():
    torch.manual_seed(0)
    m = MLP()
    m2 = copy.deepcopy(m)
    o = SGD(m.parameters(), 0.05, momentum=0.9, weight_decay=1e-4)
    o2 = torch.optim.SGD(m2.parameters(), 0.05, momentum=0.9, weight_decay=1e-4)
    for _ in range(5):
        x = torch.randn(8, 16)
        y = torch.randint(0, 8, (8,))
        o.zero_grad()
        MF.cross_entropy(m(x), y).backward()
        o.step()
        o2.zero_grad()
        torch.nn.functional.cross_entropy(m2(x), y).backward()
        o2.step()
    for p, q in zip(m.parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=1e-6)
    # flat storage: params are views of one buffer, grads of another
    sp = flat_space_for(m.fc1.weight)
    assert sp is not None and m.fc1.weight.data_ptr() >= sp.flat.data_ptr()
    o2.load_state_dict(o.state_dict())
    o.load_state_dict(o2.state_dict())


def test_adamw_matches_torch():
    torch.manual_seed(0)
    m = MLP()
    m2 = copy.deepcopy(m)
    o = AdamW(m.parameters(), 1e-2, weight_decay=0.01)
    o2 = torch.optim.AdamW(m2.parameters(), 1e-2, weight_decay=0.01)
    for _ in range(4):
        x = torch.randn(8, 16)
        y = torch.randint(0, 8, (8,))
        o.zero_grad()
        MF.cross_entropy(m(x), y).backward()
        o.step()
        o2.zero_grad()
        torch.nn.functional.cross_entropy(m2(x), y).backward()
        o2.step()
    for p, q in zip(m.parameters(), m2.parameters()):
        assert torch.allclose(p, q, atol=1e-5)


def _ddp_worker(rank, world, port, out, check_mismatch, double_report=False):
    import torch.distributed as dist
    from mipipe.parallel import DistributedDataParallel, CollectiveSequenceError
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank)  # different init per rank: DDP must broadcast rank 0's
    m = MLP()
    cap, first = (1.0, 1.0) if double_report else (0.0005, 0.0001)  # one multi-param bucket
    ddp = DistributedDataParallel(m, bucket_cap_mb=cap, first_bucket_mb=first,
                                  check_collectives=True, check_every=1)
    opt = SGD(ddp.parameters(), 0.1, momentum=0.9)
    if double_report:
        # what a kernel writing a gradient straight into the flat buffer does (space listener)
        # on top of autograd's post-accumulate hook: readiness must be counted once per step
        for p in m.parameters():
            p.register_post_accumulate_grad_hook(lambda q: ddp.space.grad_ready(q))
    g = torch.Generator().manual_seed(123)
    X = torch.randn(4 * world, 16, generator=g)
    Y = torch.randint(0, 8, (4 * world,), generator=g)
    for _ in range(3):
        opt.zero_grad()
        xs, ys = X[rank * 4:(rank + 1) * 4], Y[rank * 4:(rank + 1) * 4]
        MF.cross_entropy(ddp(xs), ys).backward()
        opt.step()
    flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    ok = True
    if check_mismatch:
        try:
            if rank == 0:  # a collective only rank 0 issues -> digest mismatch
                ddp._clog.record("broadcast", torch.zeros(3))
            ddp.verify_collective_sequence()
            ok = False
        except CollectiveSequenceError:
            ok = True
    out[rank] = (flat, len(ddp.buckets), ok)
    dist.destroy_process_group()


@pytest.mark.parametrize("double_report", [False, True])
def test_ddp_gloo_matches_single_process(double_report):
    world = 2
    port = 29000 + os.getpid() % 1000 + (500 if double_report else 0)
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_ddp_worker, args=(world, port, out, True, double_report), nprocs=world, join=True)
    f0, nb, ok0 = out[0]
    f1, _, ok1 = out[1]
    assert torch.allclose(f0, f1), "replicas diverged"
    assert nb > 1 or double_report, "expected several buckets"
    assert ok0 and ok1, "collective checker missed a mismatched sequence"
    # single process on the global batch, starting from rank 0's init
    torch.manual_seed(0)
    m = MLP()
    opt = SGD(m.parameters(), 0.1, momentum=0.9)
    g = torch.Generator().manual_seed(123)
    X = torch.randn(4 * world, 16, generator=g)
    Y = torch.randint(0, 8, (4 * world,), generator=g)
    for _ in range(3):
        opt.zero_grad()
        MF.cross_entropy(m(X), Y).backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert torch.allclose(f0, ref, atol=1e-5)


@pytest.mark.parametrize("reducer", ["python", "native"])
def test_ddp_check_tool_cpu(reducer):
    """tools/ddp_gpu_check.py on the CPU path (2 gloo ranks).  Python reducer: bucket all-reduces
    intercepted -- no gradient lands after its bucket launched, reduced == sum of local gradients.
    Native reducer (mipipe._C.Reducer): the collectives are issued from C++; the all-reduced
    gradient is checked against single-process replicas.  Both: the ranks stay bit-identical."""
    if reducer == "native":
        from mipipe.ops._native import native_available
        if not native_available():
            pytest.skip("mipipe._C not built")
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    port = str(29100 + os.getpid() % 800)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port", port,
                        os.path.join(root, "tools", "ddp_gpu_check.py"), "--device", "cpu",
                        "--arch", "resnet18", "--reducer", reducer], capture_output=True,
                       text=True, timeout=600, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    first = "step0 bucket check OK" if reducer == "python" else "step0 native reducer"
    assert first in r.stdout and "DDP gpu check OK" in r.stdout
    assert "step0 gradient vs truth" in r.stdout


def test_data_parallel_passthrough_and_unwrap():
    """DataParallel (reference task.py:201-208 path (d)) with <= 1 device is a pass-through, and
    task.py's unwrap returns the inner module (so evaluation and export see torchvision keys)."""
    from mipipe.parallel import DataParallel
    from mipipe.train.task import _unwrap
    torch.manual_seed(0)
    inner = torch.nn.Sequential(torch.nn.Linear(8, 4), torch.nn.ReLU(), torch.nn.Linear(4, 3))
    dp = DataParallel(inner)
    x = torch.randn(5, 8)
    torch.testing.assert_close(dp(x), inner(x))
    assert _unwrap(dp) is inner
    assert set(inner.state_dict()) == set(_unwrap(dp).state_dict())


def _bucket_layout_worker(rank, world, port, out):
    import torch.distributed as dist
    from mipipe.models import create_model
    from mipipe.parallel import DistributedDataParallel
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    d = DistributedDataParallel(create_model("resnet50", num_classes=1000), force_reduce=True)
    out[rank] = [(b.start, b.end, len(b.params)) for b in d.buckets]
    dist.destroy_process_group()


def test_ddp_bucket_layout_small_tail():
    """ResNet-50 buckets: contiguous slices covering the flat gradient buffer, a small first
    bucket (classifier), a small LAST bucket (stem + first layer: the all-reduce left exposed
    after the final backward kernel) and middle buckets within the cap."""
    out = mp.Manager().dict()
    mp.spawn(_bucket_layout_worker, args=(1, 29300 + os.getpid() % 500, out), nprocs=1)
    b = out[0]
    assert b[0][0] == 0
    assert all(b[k][1] == b[k + 1][0] for k in range(len(b) - 1))
    mb = [(e - s) * 4 / 2 ** 20 for s, e, _ in b]
    assert mb[-1] <= 4.0 and mb[0] <= 10.0, mb
    assert all(m <= 32.0 for m in mb[1:-1]), mb
    assert len(b) >= 4


def _bert_bucket_worker(rank, world, port, out):
    import copy
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mipipe.models import create_model
    from mipipe.parallel import DistributedDataParallel
    torch.manual_seed(0)
    m = create_model("bert_base", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    ref = copy.deepcopy(m)
    d = DistributedDataParallel(m, force_reduce=True)
    wte = m.bert.embeddings.word_embeddings.weight
    res = {"buckets": [(b.start, b.end, len(b.params)) for b in d.buckets],
           "first_is_wte": d.buckets[0].params[0] is wte and len(d.buckets[0].params) == 1,
           "sparse": len(d._sparse)}
    # one step: the DDP gradient (dense part all-reduced in bucket 0, lookup rows all-gathered
    # and scattered in order) equals the plain model's
    B, S, P = 2, 16, 3
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(0, 30522, (B, S), generator=g)
    ids[:, :4] = 7  # repeated tokens
    am = torch.ones(B, S, dtype=torch.int64)
    pos = torch.stack([torch.randperm(S, generator=g)[:P] for _ in range(B)])
    lab = torch.randint(0, 30522, (B, P), generator=g)
    d(ids, am, masked_positions=pos, labels=lab).backward()
    ref(ids, am, masked_positions=pos, labels=lab).backward()
    res["sent_bytes"] = d._sparse[0].sent_bytes
    errs = []
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        if not torch.allclose(p.grad, q.grad, rtol=1e-4, atol=1e-6):
            errs.append((n, float((p.grad - q.grad).abs().max())))
    res["grad_errs"] = errs
    out[rank] = res
    dist.destroy_process_group()


def test_ddp_bert_tied_embedding_not_exposed():
    """BERT-base: the tied word embedding's 94 MB gradient no longer sits in the last bucket.
    Its dense (decoder) part is reduced in bucket 0 — ready at the start of the backward — and
    its lookup part is exchanged as (id, row) pairs.  What is left after the last backward kernel
    is the last bucket + those pairs: <= 8 MB per rank at 32 x 128 tokens (bf16 rows on the GPU).
    The DDP gradient equals the plain model's (world 1, gloo)."""
    out = mp.Manager().dict()
    mp.spawn(_bert_bucket_worker, args=(1, 29350 + os.getpid() % 400, out), nprocs=1)
    r = out[0]
    assert r["first_is_wte"] and r["sparse"] == 1
    b = r["buckets"]
    assert b[0][0] == 0 and all(b[k][1] == b[k + 1][0] for k in range(len(b) - 1))
    last_mb = (b[-1][1] - b[-1][0]) * 4 / 2 ** 20
    tokens, H = 32 * 128, 768
    pairs_mb = (tokens * H * 2 + tokens * 8) / 2 ** 20  # bf16 rows + int64 ids
    assert last_mb + pairs_mb <= 8.0, (last_mb, pairs_mb)
    assert r["sent_bytes"] == 2 * 16 * (768 * 4 + 8)  # this CPU step: fp32 rows + ids
    assert not r["grad_errs"], r["grad_errs"]


def _ids_in_forward_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mipipe.models import create_model
    from mipipe.parallel import DistributedDataParallel
    torch.manual_seed(0)
    m = create_model("bert_tiny", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    d = DistributedDataParallel(m)
    ex = d._sparse[0]
    V = m.bert.embeddings.word_embeddings.weight.shape[0]
    res = {}

    def batch(B, S, seed):
        g = torch.Generator().manual_seed(seed)
        ids = torch.randint(0, V, (B, S), generator=g)
        ids[:, :S // 2] = 0  # a [PAD]-like run: one id repeated across many chunks
        am = torch.ones(B, S, dtype=torch.int64)
        pos = torch.stack([torch.randperm(S, generator=g)[:3] for _ in range(B)])
        lab = torch.randint(0, V, (B, 3), generator=g)
        return ids, am, pos, lab

    ids, am, pos, lab = batch(4, 32, 10 + rank)
    loss = d(ids, am, masked_positions=pos, labels=lab)
    # the ids' all_gather was issued by the forward and already sorted: before backward()
    res["issued_before_backward"] = (ex.fwd is not None and ex.fwd["sorted"] is not None
                                     and ex.ids_issued_in_forward == 1)
    loss.backward()
    res["cap"] = ex.cap
    # ragged step (fewer tokens on rank 1): padded to the agreed capacity, same collectives
    B = 4 if rank == 0 else 3
    ids, am, pos, lab = batch(B, 32, 20 + rank)
    d.zero_grad() if hasattr(d, "zero_grad") else None
    d(ids, am, masked_positions=pos, labels=lab).backward()
    res["ragged_ok"] = ex.ids_issued_in_forward == 2
    wg = m.bert.embeddings.word_embeddings.weight.grad.clone()
    gathered = [torch.zeros_like(wg) for _ in range(world)]
    dist.all_gather(gathered, wg)
    res["same_on_all_ranks"] = all(torch.equal(gathered[0], x) for x in gathered)
    # more tokens than the capacity: a clear error before any collective
    try:
        ids, am, pos, lab = batch(5, 32, 30)
        d(ids, am, masked_positions=pos, labels=lab)
        res["grow_raises"] = False
    except RuntimeError as e:
        res["grow_raises"] = "capacity" in str(e)
    out[rank] = res
    dist.destroy_process_group()


def test_ddp_bert_lookup_ids_exchanged_during_forward():
    """World 4 (gloo): the tied word embedding's lookup ids are all-gathered and stably sorted
    during the FORWARD (SURVEY §2.6 C5''): after the last backward kernel only the rows' gather
    and the scatter remain.  A ragged step with fewer tokens on one rank is padded to the
    capacity agreed at the first step (same collectives on every rank, identical gradients);
    more tokens than the capacity raises instead of mismatching the collective."""
    out = mp.Manager().dict()
    mp.spawn(_ids_in_forward_worker, args=(4, 29400 + os.getpid() % 400, out), nprocs=4)
    for r in range(4):
        assert out[r]["issued_before_backward"], out[r]
        assert out[r]["cap"] == 4 * 32
        assert out[r]["ragged_ok"] and out[r]["same_on_all_ranks"], out[r]
        assert out[r]["grow_raises"], out[r]


def _one_rank_grows_worker(rank, world, port, out):
    import datetime
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=30))
    from mipipe.models import create_model
    from mipipe.parallel import DistributedDataParallel
    torch.manual_seed(0)
    m = create_model("bert_tiny", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    d = DistributedDataParallel(m)
    V = m.bert.embeddings.word_embeddings.weight.shape[0]

    def batch(B, S=16):
        g = torch.Generator().manual_seed(rank)
        return (torch.randint(0, V, (B, S), generator=g), torch.ones(B, S, dtype=torch.int64),
                torch.zeros(B, 2, dtype=torch.int64), torch.randint(0, V, (B, 2), generator=g))

    ids, am, pos, lab = batch(2)
    d(ids, am, masked_positions=pos, labels=lab).backward()
    res = {"cap": d._sparse[0].cap}
    # only rank 1 grows: it raises before issuing; rank 0 must not complete the step silently
    ids, am, pos, lab = batch(3 if rank == 1 else 2)
    try:
        d(ids, am, masked_positions=pos, labels=lab).backward()
        res["outcome"] = "completed"
    except RuntimeError as e:
        res["outcome"] = "capacity" if "capacity" in str(e) else "peer_error"
    out[rank] = res
    # no destroy_process_group: the group is broken by design here; the process exit closes it


def test_ddp_sparse_capacity_one_rank_grows():
    """Only ONE rank exceeds the agreed capacity (advice r5): that rank raises the capacity
    error before any collective and its peer's pending ids all_gather fails (peer closed /
    timeout) — neither rank completes a step with a mismatched collective."""
    out = mp.Manager().dict()
    mp.spawn(_one_rank_grows_worker, args=(2, 29800 + os.getpid() % 150, out), nprocs=2)
    assert out[1]["outcome"] == "capacity", dict(out)
    assert out[0]["outcome"] == "peer_error", dict(out)
    assert out[0]["cap"] == out[1]["cap"] == 2 * 16
