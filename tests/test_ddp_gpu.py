"""DDP over RCCL on one MI355X: the nccl(=RCCL) backend at world size 1 with ``force_reduce``
issues every collective the multi-GPU run issues (construction broadcast, per-forward buffer
broadcast, bucketed gradient all-reduce overlapped with backward), and a hipGraph capture of
the whole DDP step (collectives included) replays the same training math as eager steps.

Reference contract: task.py:148-149 (init_process_group nccl), :189 (DDP(model,
device_ids=[gpu])), :309-312 (the step)."""
import copy
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cos(a, b):
    a = a.detach().float().flatten()
    b = b.detach().float().flatten()
    return float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))


@pytest.fixture(scope="module")
def nccl_pg():
    import torch.distributed as dist
    from mipipe.launch.launcher import free_port
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{free_port()}", rank=0,
                            world_size=1, device_id=torch.device("cuda", 0))
    yield dist
    dist.destroy_process_group()


def test_rccl_ddp_graphed_matches_eager(nccl_pg):
    """DDP (RCCL, world 1, every bucket forced through the collective) replayed from a hipGraph
    == the same steps run eagerly.  Deterministic kernels: without them a batch-32 bf16
    BatchNorm net amplifies atomic-order noise to ~0.98 cosine between two EAGER runs within
    four SGD steps, which is no basis for comparing graph against eager."""
    from mipipe.models import create_model
    from mipipe.ops.determinism import deterministic
    from mipipe.ops.functional import cross_entropy
    from mipipe.optim import SGD
    from mipipe.parallel import DistributedDataParallel
    from mipipe.train.graph import GraphedStep, graph_safe
    torch.manual_seed(0)
    base = create_model("resnet18", num_classes=10).cuda()
    mods = [copy.deepcopy(base) for _ in range(2)]
    ddps = [DistributedDataParallel(m, device_ids=[0], force_reduce=True, bucket_cap_mb=8)
            for m in mods]
    for d in ddps:
        assert d._comm and len(d.buckets) >= 2
    opts = [SGD(d.parameters(), 0.05, momentum=0.9, weight_decay=1e-4) for d in ddps]
    assert graph_safe(ddps[1], opts[1])[0]
    x = torch.randn(32, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (32,), device="cuda")

    def make_step(m, o):
        def step(xx, yy):
            o.zero_grad()
            loss = cross_entropy(m(xx), yy)
            loss.backward()
            o.step()
            return loss
        return step

    with deterministic(True):
        la = [make_step(ddps[0], opts[0])(x, y).item() for _ in range(4)]
        n0 = ddps[0]._clog.count
        # per eager step: one buffer broadcast per dtype + one all-reduce per bucket
        assert n0 >= 4 * len(ddps[0].buckets)
        c0 = ddps[1]._clog.count
        gs = GraphedStep(make_step(ddps[1], opts[1]), (x, y), warmup=1, inputs=[(x, y)])
        assert ddps[1]._clog.count - c0 >= 2 * len(ddps[1].buckets)  # eager warmup + capture
        lb = [gs.replay(0).item() for _ in range(3)]
        torch.cuda.synchronize()
    assert abs(la[-1] - lb[-1]) <= 1e-5 * abs(la[-1]), (la, lb)
    for (n, p), (_, q) in zip(mods[0].named_parameters(), mods[1].named_parameters()):
        assert cos(p, q) > 0.99999, (n, cos(p, q))
    for (n, b), (_, c) in zip(mods[0].named_buffers(), mods[1].named_buffers()):
        if b.is_floating_point():
            torch.testing.assert_close(b, c, rtol=1e-4, atol=1e-5, msg=n)

def test_rccl_bf16_comm_dtype(nccl_pg):
    """comm_dtype=bf16 halves the bytes on the wire; the averaged gradient equals the fp32
    gradient to bf16 rounding."""
    from mipipe.models import create_model
    from mipipe.ops.functional import cross_entropy
    from mipipe.parallel import DistributedDataParallel
    torch.manual_seed(1)
    m = create_model("resnet18", num_classes=10).cuda()
    d = DistributedDataParallel(m, device_ids=[0], force_reduce=True, comm_dtype=torch.bfloat16)
    x = torch.randn(16, 3, 32, 32, device="cuda")
    y = torch.randint(0, 10, (16,), device="cuda")
    d.space.zero_grad()
    cross_entropy(d(x), y).backward()
    g = d.space.flat_grad.clone()
    assert torch.isfinite(g).all() and g.abs().sum() > 0
    # every bucket went through a bf16 temporary: values are bf16-representable
    assert torch.equal(g, g.to(torch.bfloat16).float())


def test_bench_force_reduce_graph_gpu():
    """bench.py with --force-reduce: DDP + RCCL + hipGraph replay in the timed loop."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="0", WORLD_SIZE="1", RANK="0", LOCAL_RANK="0",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1",
                        "--force-reduce", "--model", "resnet18", "--res", "32", "--batch", "128",
                        "--steps", "5", "--warmup", "2"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    j = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][0]
    assert j["config"]["hip_graph"] is True and j["config"]["force_reduce"] is True
    assert j["value"] > 0 and j["final_loss"] == j["final_loss"]
