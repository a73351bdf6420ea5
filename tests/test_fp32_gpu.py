"""fp32 (the reference's precision, task.py:303-312 has no autocast) on the gfx950 kernels.

GEMM-shaped kernels run the split-bf16x3 main loop (fp32 operands split exactly into three bf16
parts in LDS, 6 MFMAs per tile, fp32 accumulation); elementwise / reduction kernels read and
write fp32.  Every kernel is compared against a float64 evaluation of the same op on the same
fp32 inputs; the bound is 1e-4 relative to the output magnitude (measured ~1e-6, like stock
fp32 torch; bf16 would be ~1e-2).
"""
import math

import pytest
import torch

from mipipe.ops import _ref
from mipipe.ops._native import native, native_available

pytestmark = pytest.mark.gpu

dev = "cuda"
TOL = 1e-4


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_available(), "mipipe._C must be built for GPU tests (no silent fallback)"
    torch.manual_seed(4321)
    yield


def rel_err(a, b):
    a = a.double().cpu()
    b = b.double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-12)).item()


def f32(*shape, scale=1.0):
    return torch.randn(*shape, device=dev) * scale


def d(t):
    return t.detach().double().cpu()


# ResNet-18 on 32x32 inputs (the reference's CIFAR config of record) layer shapes, batch 32,
# plus odd / strided / 7x7 cases.  N, H, W, Ci, Co, k, s, p
CONV_CASES = [
    (32, 16, 16, 8, 64, 3, 1, 1),
    (32, 8, 8, 64, 64, 3, 1, 1),
    (32, 8, 8, 64, 128, 3, 2, 1),
    (32, 8, 8, 64, 128, 1, 2, 0),
    (32, 4, 4, 128, 128, 3, 1, 1),
    (32, 4, 4, 128, 256, 3, 2, 1),
    (32, 2, 2, 256, 512, 3, 2, 1),
    (32, 1, 1, 512, 512, 3, 1, 1),
    (4, 14, 14, 256, 1024, 1, 1, 0),
    (2, 9, 7, 32, 72, 3, 1, 1),
    (2, 32, 32, 8, 64, 7, 2, 3),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_fp32(case):
    N, H, W, Ci, Co, k, s, p = case
    x = f32(N, H, W, Ci)
    w = f32(Co, k, k, Ci, scale=1.0 / math.sqrt(Ci * k * k))
    shift = torch.randn(Co, device=dev) * 0.1
    y, ps, pss = native().conv_fwd(x, w, s, p, shift)
    assert y.dtype == torch.float32
    yr, psr, pssr = _ref.conv_fwd(d(x), d(w), s, p, d(shift))
    assert rel_err(y, yr) < TOL
    assert rel_err(ps.sum(0), psr[0]) < TOL
    assert rel_err(pss.sum(0), pssr[0]) < TOL


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad_fp32(case):
    N, H, W, Ci, Co, k, s, p = case
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = f32(N, Ho, Wo, Co)
    w = f32(Co, k, k, Ci, scale=1.0 / math.sqrt(Co * k * k))
    dx = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p)
    assert dx.dtype == torch.float32
    assert rel_err(dx, _ref.conv_dgrad(d(dy), d(w), (N, H, W, Ci), s, p)) < TOL


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_wgrad_fp32(case):
    N, H, W, Ci, Co, k, s, p = case
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = f32(N, Ho, Wo, Co)
    x = f32(N, H, W, Ci)
    dw = native().conv_wgrad(dy, x, k, k, s, p)
    assert rel_err(dw, _ref.conv_wgrad(d(dy), d(x), k, k, s, p)) < TOL


def test_conv_dgrad_fused_epilogue_fp32():
    # dgrad of a conv whose input was relu(bn(y)) + a residual addend: fp32 epilogue fusions
    N, H, W, Ci, Co = 8, 8, 8, 64, 64
    dy = f32(N, H, W, Co)
    w = f32(Co, 3, 3, Ci, scale=1.0 / math.sqrt(Co * 9))
    y = f32(N, H, W, Ci)
    add = f32(N, H, W, Ci)
    mean = torch.randn(Ci, device=dev) * 0.1
    invstd = torch.rand(Ci, device=dev) + 0.5
    gamma = torch.rand(Ci, device=dev) + 0.5
    beta = torch.randn(Ci, device=dev) * 0.1
    scale, bias = gamma * invstd, beta - mean * gamma * invstd
    rep = torch.zeros(3, native().STAT_REPLICAS, Ci, device=dev)
    g = native().conv_dgrad(dy, w, [N, H, W, Ci], 1, 1, add, y, mean, invstd, scale, bias, rep)
    sg, sgx = native().bn_bwd_collect(rep, Ci)
    dx = _ref.conv_dgrad(d(dy), d(w), (N, H, W, Ci), 1, 1) + d(add)
    z = d(y) * d(scale) + d(bias)
    gr = dx * (z > 0)
    assert rel_err(g, gr) < TOL
    xhat = (d(y) - d(mean)) * d(invstd)
    assert rel_err(sg, gr.reshape(-1, Ci).sum(0)) < TOL
    assert rel_err(sgx, (gr * xhat).reshape(-1, Ci).sum(0)) < TOL


def test_conv_dgrad_fused_bn_sums_fp32_large_mean():
    """fp32 BN-backward sums at |mean| >> std (advice r5): the fp32 epilogue accumulates the
    centred g·(y - mean)·invstd — the uncentred invstd·(Σg·y - mean·Σg) form the bf16 path uses
    would cancel ~|mean|/std = 1e3 of its digits here."""
    N, H, W, Ci, Co = 8, 8, 8, 64, 64
    dy = f32(N, H, W, Co)
    w = f32(Co, 1, 1, Ci, scale=1.0 / math.sqrt(Co))
    y = 50.0 + 0.05 * f32(N, H, W, Ci)
    mean = y.double().reshape(-1, Ci).mean(0).float()
    invstd = (1.0 / y.double().reshape(-1, Ci).std(0, unbiased=False)).float()
    gamma = torch.rand(Ci, device=dev) + 0.5
    beta = torch.full((Ci,), 10.0, device=dev)  # z = γx̂ + β > 0: no ReLU decision near 0
    scale, bias = gamma * invstd, beta - mean * gamma * invstd
    rep = torch.zeros(3, native().STAT_REPLICAS, Ci, device=dev)
    g = native().conv_dgrad(dy, w, [N, H, W, Ci], 1, 0, None, y, mean, invstd, scale, bias, rep)
    sg, sgx = native().bn_bwd_collect(rep, Ci)
    gr = _ref.conv_dgrad(d(dy), d(w), (N, H, W, Ci), 1, 0) * ((d(y) * d(scale) + d(bias)) > 0)
    assert rel_err(g, gr) < TOL
    xhat = (d(y) - d(mean)) * d(invstd)
    assert rel_err(sg, gr.reshape(-1, Ci).sum(0)) < TOL
    assert rel_err(sgx, (gr * xhat).reshape(-1, Ci).sum(0)) < TOL


@pytest.mark.parametrize("M,N,K", [(1024, 512, 512), (300, 72, 200), (32, 1000, 512),
                                   (1024, 10, 512)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
def test_gemm_fp32(M, N, K, ta, tb):
    if (ta and M % 8) or (not ta and K % 8) or N % 8 or (tb and K % 8):
        pytest.skip("layout constraint")
    a = f32(K, M) if ta else f32(M, K)
    b = f32(N, K) if tb else f32(K, N)
    bias = torch.randn(N, device=dev)
    out = native().gemm(a, b, ta, tb, bias, "relu", torch.float32, None, 0.0)
    ref = _ref.gemm(d(a), d(b), ta, tb, d(bias), "relu", torch.float64)
    assert out.dtype == torch.float32 and rel_err(out, ref) < TOL
    acc = torch.randn(M, N, device=dev)
    acc0 = d(acc)
    native().gemm(a, b, ta, tb, None, "none", torch.float32, acc, 1.0)
    assert rel_err(acc, acc0 + _ref.gemm(d(a), d(b), ta, tb, None, "none", torch.float64)) < TOL


@pytest.mark.parametrize("C", [64, 512])
def test_bn_kernels_fp32(C):
    M = 32 * 8 * 8
    y = f32(M, C) * 2 + 0.5
    dz = f32(M, C)
    res = f32(M, C)
    mean = d(y).mean(0)
    var = d(y).var(0, unbiased=False)
    invstd = torch.rsqrt(var + 1e-5)
    gamma = torch.rand(C, dtype=torch.float64) + 0.5
    beta = torch.randn(C, dtype=torch.float64) * 0.1
    scale, bias = gamma * invstd, beta - mean * gamma * invstd
    g32 = lambda t: t.float().to(dev)  # noqa: E731
    z = native().bn_act_fwd(y, g32(scale), g32(bias), True, res, None, None)
    zr = _ref.bn_act_fwd(d(y), scale, bias, True, d(res))
    assert z.dtype == torch.float32 and rel_err(z, zr) < TOL
    sg, sgx, _ = native().bn_act_bwd_reduce(dz, z, y, g32(mean), g32(invstd), True)
    sgr, sgxr = _ref.bn_act_bwd_reduce(d(dz), zr, d(y), mean, invstd, True)
    assert rel_err(sg, sgr) < TOL and rel_err(sgx, sgxr) < TOL
    dy, dres = native().bn_act_bwd_apply(dz, z, y, g32(mean), g32(invstd), g32(gamma), sg, sgx,
                                         M, True, True, None, None, None, None, None)
    dyr, dresr = _ref.bn_act_bwd_apply(d(dz), zr, d(y), mean, invstd, gamma, sgr, sgxr, M, True,
                                       True)
    assert rel_err(dy, dyr) < TOL and rel_err(dres, dresr) < TOL


def test_pools_fp32():
    x = f32(32, 16, 16, 64)
    y, idx = native().maxpool_fwd(x, 3, 2, 1)
    yr, _ = _ref.maxpool_fwd(d(x), 3, 2, 1)
    assert y.dtype == torch.float32 and torch.equal(y.cpu().double(), yr)
    dy = f32(*y.shape)
    dx = native().maxpool_bwd_impl(dy, idx, list(x.shape), 3, 2, 1)
    xr = d(x).permute(0, 3, 1, 2).requires_grad_(True)
    torch.nn.functional.max_pool2d(xr, 3, 2, 1).backward(d(dy).permute(0, 3, 1, 2))
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < TOL
    a = native().avgpool_fwd(x)
    assert rel_err(a, _ref.avgpool_fwd(d(x))) < TOL
    da = f32(32, 64)
    assert rel_err(native().avgpool_bwd(da, list(x.shape)), _ref.avgpool_bwd(d(da), x.shape)) < TOL


@pytest.mark.parametrize("V", [10, 1000])
def test_cross_entropy_fp32(V):
    logits = f32(256, V) * 3
    labels = torch.randint(0, V, (256,), device=dev)
    loss, grad = native().cross_entropy_fwd_bwd(logits, labels, 0.0, -100)
    lr, gr = _ref.cross_entropy_fwd_bwd(d(logits), labels.cpu())
    assert grad.dtype == torch.float32
    assert abs(loss.item() - lr.item()) / abs(lr.item()) < TOL
    assert rel_err(grad, gr) < TOL


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("V", [10, 1000])
def test_top1_correct(dtype, V):
    R = 777
    logits = f32(R, V).to(dtype)
    logits[::7, 3] = logits[::7].float().max(1).values.to(dtype)  # ties: first index wins
    labels = torch.randint(0, V, (R,), device=dev)
    labels[::5] = logits[::5].float().argmax(1)
    out = torch.zeros(1, dtype=torch.int32, device=dev)
    native().top1_correct(logits, labels, out)
    native().top1_correct(logits, labels, out)
    ref = (logits.float().argmax(1) == labels).sum().item()
    assert out.item() == 2 * ref


def test_layout_kernels_fp32():
    x = torch.rand(8, 3, 32, 32, device=dev)
    y = native().nchw_to_nhwc(x, torch.float32, 8)
    assert y.dtype == torch.float32 and torch.equal(y[..., :3], x.permute(0, 2, 3, 1))
    assert torch.count_nonzero(y[..., 3:]) == 0
    p = native().stem_pack(x, 3, 37, 19, torch.float32)[0]
    pb = native().stem_pack(x, 3, 37, 19, torch.bfloat16)[0]
    assert p.dtype == torch.float32 and rel_err(p, pb.float()) < 1e-2


@pytest.mark.parametrize("det", [False, True], ids=["default", "deterministic"])
def test_resnet18_cifar_fp32_step_matches_float64(det):
    """One ResNet-18 (32x32, 10 classes, batch 64) fwd + bwd in fp32 on the HIP kernels vs a
    float64 evaluation of the same weights and inputs that takes every ReLU / max-pool DECISION
    from the GPU run (tests/pinned_ref.py).  Round 4's driver box saw one tensor at 1.16e-2
    relative L2 against an unpinned float64 reference: a ReLU pre-activation within fp32
    rounding of 0 (atomics order in the BN statistics moves which ones) decides differently and
    moves a small layer-4 BatchNorm gradient by ~1/64.  With decisions pinned, what is left is
    arithmetic, and every tensor must be within 1e-4 in both modes (default = fp32 atomics in the
    BN statistics / split-K; deterministic = fixed-order sums, task.py:25)."""
    from mipipe.models import create_model
    from mipipe.ops.determinism import deterministic
    from mipipe.train.task import CrossEntropyLoss
    from pinned_ref import flipped_decisions, pinned_grads, record_gpu_decisions
    torch.manual_seed(0)
    m = create_model("resnet18", num_classes=10)
    state = {k: v.clone() for k, v in m.state_dict().items()}
    names = [n for n, _ in m.named_parameters()]
    m = m.to(dev)
    m.compute_dtype = torch.float32
    x = torch.randn(64, 3, 32, 32)
    yl = torch.randint(0, 10, (64,))
    with deterministic(det), record_gpu_decisions() as tape:
        out = m(x.to(dev))
        loss = CrossEntropyLoss()(out, yl.to(dev))
        loss.backward()
    torch.cuda.synchronize()
    assert len(tape.relu_masks) == 16 and tape.pool is not None, tape.summary()
    out_r, loss_r, g_pin, _ = pinned_grads(state, names, x, yl, tape)
    _, _, g_own, pin_own = pinned_grads(state, names, x, yl, None)
    flips = flipped_decisions(tape, pin_own.own)
    assert out.dtype == torch.float32
    assert rel_err(out, out_r) < 1e-4
    assert abs(loss.item() - loss_r.item()) < 1e-5 * max(1.0, abs(loss_r.item()))
    grads = dict(m.named_parameters())

    def rl2(a, b):
        return ((a.double().cpu() - b).norm() / b.norm()).item()
    pinned = sorted(((rl2(grads[n].grad, g_pin[n]), n) for n in names), reverse=True)
    unpinned = sorted(((rl2(grads[n].grad, g_own[n]), n) for n in names), reverse=True)
    report = (f"decisions flipped vs float64: {flips or 'none'}; worst pinned: {pinned[:4]}; "
              f"worst unpinned: {unpinned[:4]}")
    print(report)
    assert all(e < 1e-4 for e, _ in pinned), report


# vision.hip kernels (grouped / depthwise / non-square direct conv, any-C BatchNorm, k x k avg
# pool) in fp32: N, H, W, Ci, Co, (kh, kw), (sh, sw), (ph, pw), groups
GCONV_CASES = [
    (2, 14, 14, 96, 96, (3, 3), (1, 1), (1, 1), 96),
    (2, 9, 9, 40, 40, (5, 5), (2, 2), (2, 2), 40),
    (2, 7, 7, 58, 58, (3, 3), (1, 1), (1, 1), 58),
    (2, 8, 8, 128, 128, (3, 3), (2, 2), (1, 1), 32),
    (2, 9, 11, 64, 48, (1, 7), (1, 1), (0, 3), 1),
]


@pytest.mark.parametrize("case", GCONV_CASES)
def test_gconv_fp32(case):
    N, H, W, Ci, Co, k, s, p, g = case
    x = f32(N, H, W, Ci)
    w = f32(Co, k[0], k[1], Ci // g, scale=1.0 / math.sqrt(Ci // g * k[0] * k[1]))
    b = torch.randn(Co, device=dev) * 0.1
    y = native().gconv_fwd(x, w, list(s), list(p), g, b, 2)
    assert y.dtype == torch.float32
    assert rel_err(y, _ref.gconv_fwd(d(x), d(w), s, p, g, d(b), "relu6")) < TOL
    dy = f32(*y.shape)
    dx = native().gconv_dgrad(dy, w, [N, H, W, Ci], list(s), list(p), g, y, 2)
    assert rel_err(dx, _ref.gconv_dgrad(d(dy), d(w), (N, H, W, Ci), s, p, g, d(y), "relu6")) < TOL
    dw, db = native().gconv_wgrad(dy, x, k[0], k[1], list(s), list(p), g, y, 2, None, None, True)
    dwr, dbr = _ref.gconv_wgrad(d(dy), d(x), k[0], k[1], s, p, g, d(y), "relu6")
    assert rel_err(dw, dwr) < TOL and rel_err(db, dbr) < TOL


@pytest.mark.parametrize("C", [58, 96])
def test_bn_generic_and_avgpool2d_fp32(C):
    y = f32(3, 7, 9, C) * 2 + 0.5
    shift = torch.randn(C, device=dev) * 0.1
    ps, pq = native().chan_stats(y, shift)
    assert ps.shape[0] == native().STAT_REPLICAS  # replica rows, summed by bn_finalize
    psr, pqr = _ref.chan_stats(d(y), d(shift))
    ps, pq = ps.sum(0).reshape(psr.shape), pq.sum(0).reshape(pqr.shape)
    assert rel_err(ps, psr) < TOL and rel_err(pq, pqr) < TOL
    scale, bias = torch.randn(C, device=dev), torch.randn(C, device=dev)
    z = native().affine_act(y, scale, bias, 1)
    assert z.dtype == torch.float32
    assert rel_err(z, _ref.affine_act(d(y), d(scale), d(bias), "relu")) < TOL
    mean, invstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    gamma = torch.randn(C, device=dev)
    dz = f32(*y.shape)
    sg, sgx = native().bn_generic_bwd_reduce(dz, z, y, mean, invstd, 1)
    sgr, sgxr = _ref.bn_generic_bwd_reduce(d(dz), d(z), d(y), d(mean), d(invstd), "relu")
    assert rel_err(sg, sgr) < TOL and rel_err(sgx, sgxr) < TOL
    n = y.numel() // C
    dy = native().bn_generic_bwd_apply(dz, z, y, mean, invstd, gamma, sg, sgx, n, 1)
    dyr = _ref.bn_generic_bwd_apply(d(dz), d(z), d(y), d(mean), d(invstd), d(gamma), sgr, sgxr,
                                    n, "relu")
    assert rel_err(dy, dyr) < TOL
    x = f32(2, 17, 17, C)
    a = native().avgpool2d_fwd(x, 3, 2, 1)
    assert a.dtype == torch.float32 and rel_err(a, _ref.avgpool2d_fwd(d(x), 3, 2, 1)) < TOL
    da = f32(*a.shape)
    assert rel_err(native().avgpool2d_bwd(da, list(x.shape), 3, 2, 1),
                   _ref.avgpool2d_bwd(d(da), tuple(x.shape), 3, 2, 1)) < TOL


ZOO = [("mobilenet_v2", 64), ("mnasnet1_0", 64), ("shufflenet_v2_x1_0", 64),
       ("squeezenet1_1", 64), ("densenet121", 64), ("googlenet", 64), ("inception_v3", 299),
       ("resnext50_32x4d", 64), ("vgg11_bn", 64), ("alexnet", 64)]
NODROP = {"mobilenet_v2": dict(dropout=0.0), "mnasnet1_0": dict(dropout=0.0),
          "squeezenet1_1": dict(dropout=0.0), "googlenet": dict(dropout=0.0, dropout_aux=0.0),
          "inception_v3": dict(dropout=0.0), "vgg11_bn": dict(dropout=0.0),
          "alexnet": dict(dropout=0.0)}


@pytest.mark.parametrize("arch,res", ZOO)
def test_zoo_fp32_train_step(arch, res):
    """Every zoo family trains in fp32 on the kernels (the reference's precision): the training-
    mode forward matches an fp32 torch evaluation of the same weights to fp32-class error, and
    SGD steps reduce the loss."""
    from mipipe.models import create_model
    from mipipe.optim import SGD
    from mipipe.train.task import CrossEntropyLoss
    torch.manual_seed(0)
    m = create_model(arch, num_classes=10, **NODROP.get(arch, {})).to(dev)
    m.compute_dtype = torch.float32
    x = torch.randn(8, 3, res, res, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)
    if hasattr(m, "reference_forward"):
        m.eval()
        with torch.no_grad():
            out, ref = m(x), m.reference_forward(x)
        o, r = out.double(), ref.double()
        assert out.dtype == torch.float32
        assert ((o - r).norm() / r.norm()).item() < 1e-3
        m.train()
    lr = 0.001 if arch.startswith("squeezenet") else 0.005  # no BatchNorm: smaller step
    opt = SGD(m.parameters(), lr, momentum=0.9, weight_decay=1e-4, shadow_dtype=None)
    crit = CrossEntropyLoss()
    losses = []
    for _ in range(5):
        opt.zero_grad()
        loss = crit(m(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss.item()))
    assert all(math.isfinite(v) for v in losses), losses
    assert min(losses[1:]) < losses[0], losses
