"""DataParallel([0, 0]) vs three chunked oracles on GPU (diagnostic for
tests/test_data_parallel.py): A = one module, chunk loop, one backward; B = one module, chunk
loop, one backward per chunk; C = one deep copy per chunk (what DataParallel computes)."""
import copy
import sys
import torch
sys.path.insert(0, ".")
from mipipe.models import create_model
from mipipe.optim import SGD
from mipipe.ops.functional import cross_entropy
from mipipe.ops.determinism import deterministic
import mipipe.parallel.data_parallel as D


def flat(m):
    return torch.cat([p.grad.flatten() for p in m.parameters()])


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def main(arch="resnet18", dtype=torch.bfloat16, bn_eval=False):
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    model = create_model(arch, num_classes=10).to(dev)
    model.compute_dtype = dtype
    A, B, C0, C1 = (copy.deepcopy(model) for _ in range(4))
    dp = D.DataParallel(model, device_ids=[0, 0])
    if bn_eval:
        for m in (model, A, B, C0, C1):
            for mod in m.modules():
                if isinstance(mod, torch.nn.BatchNorm2d):
                    mod.eval()
    keep = [SGD(m.parameters(), 0.05) for m in (dp, A, B, C0, C1)]
    x = torch.randn(16, 3, 32, 32, device=dev)
    y = torch.randint(0, 10, (16,), device=dev)
    xs = x.chunk(2)
    with deterministic(True):
        cross_entropy(dp(x), y).backward()
        cross_entropy(torch.cat([A(c) for c in xs]), y).backward()
        ob = [B(c) for c in xs]
        for i in range(2):
            cross_entropy(torch.cat([o if j == i else o.detach() for j, o in enumerate(ob)]), y
                          ).backward(retain_graph=True)
        oc = [C0(xs[0]), C1(xs[1])]
        cross_entropy(torch.cat(oc), y).backward()
    torch.cuda.synchronize()
    g, gA, gB = flat(model), flat(A), flat(B)
    gC = flat(C0) + flat(C1)
    print(f"DP vs A {rel(g, gA):.5f}  DP vs B {rel(g, gB):.5f}  DP vs C {rel(g, gC):.5f}")
    print(f"A vs C {rel(gA, gC):.5f}  B vs C {rel(gB, gC):.5f}  A vs B {rel(gA, gB):.5f}")
    names = [n for n, _ in model.named_parameters()]
    errs = sorted(((rel(pa.grad, pc0.grad + pc1.grad), n) for n, pa, pc0, pc1 in
                   zip(names, A.parameters(), C0.parameters(), C1.parameters())), reverse=True)
    print("  A vs C worst:", ", ".join(f"{n} {e:.3f}" for e, n in errs[:8]))
    print("  A vs C best:", ", ".join(f"{n} {e:.4f}" for e, n in errs[-4:]))
    print("replica space:", dp._rep_spaces[0] is not None,
          "replica grads drained:", float(dp._rep_spaces[0].flat_grad.abs().max()) == 0.0)
    del keep


if __name__ == "__main__":
    for kw in ({}, {"dtype": torch.float32}, {"bn_eval": True}):
        print("==", kw)
        main(**kw)
