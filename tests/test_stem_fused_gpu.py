"""Recompute-fused ResNet stem (csrc/kernels/stem.hip): conv 7x7/2 -> BN -> ReLU -> max-pool 3x3/2
without storing the conv output, against (a) the plain fp32 PyTorch reference of the same op on the
same bf16 operands and (b) the unfused kernel path (packed conv + pool_bn kernels).

Checks the pooled output, the running statistics, dW / dγ / dβ, bit-reproducibility in
deterministic mode and the eval (running-statistics) forward."""
import copy

import pytest
import torch
import torch.nn.functional as F

from mipipe import nn as mnn
from mipipe.models.resnet import _StemConv
from mipipe.ops import functional as MF
from mipipe.ops.determinism import set_deterministic
from mipipe.ops._native import native_available

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _restore():
    assert native_available()
    yield
    MF.set_stem_fused(True)
    set_deterministic(False)


def _stem(seed=0):
    torch.manual_seed(seed)
    conv = _StemConv(3, 64, kernel_size=7, stride=2, padding=3, bias=False).cuda()
    bn = mnn.BatchNorm2d(64).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        bn.running_mean.uniform_(-0.1, 0.1)
    pool = mnn.MaxPool2d(3, 2, 1)
    return conv, bn, pool


def _run(conv, bn, pool, x, dp, fused):
    MF.set_stem_fused(fused)
    xp = conv.pack_input(x, torch.bfloat16)
    out = mnn.conv_bn_relu_maxpool(xp, conv, bn, pool)
    out.backward(dp)
    torch.cuda.synchronize()
    return out


def _ref(conv, bn, x, dp):
    """fp32 PyTorch reference on the bf16-rounded operands (y, z and dy rounded where stored)."""
    xb = x.to(torch.bfloat16).float()
    w = conv.weight.detach().to(torch.bfloat16).float().requires_grad_(True)
    g = bn.weight.detach().clone().requires_grad_(True)
    b = bn.bias.detach().clone().requires_grad_(True)
    y = F.conv2d(xb, w, stride=2, padding=3)
    y.register_hook(lambda gy: gy.to(torch.bfloat16).float())  # dy is stored in bf16
    yq = y + (y.to(torch.bfloat16).float() - y).detach()  # straight-through bf16 store
    mean = yq.mean((0, 2, 3))
    var = yq.var((0, 2, 3), unbiased=False)
    z = torch.relu((yq - mean[None, :, None, None]) * torch.rsqrt(var + bn.eps)[None, :, None, None]
                   * g[None, :, None, None] + b[None, :, None, None])
    z = z + (z.to(torch.bfloat16).float() - z).detach()  # z as the kernels compare it (bf16)
    out = F.max_pool2d(z, 3, 2, 1)
    out.backward(dp.permute(0, 3, 1, 2).float())
    return out.permute(0, 2, 3, 1), w.grad, g.grad, b.grad, mean.detach(), var.detach()


def _rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("N", [2, 3])
def test_fused_stem_matches_fp32_reference(N):
    conv, bn, pool = _stem()
    g = torch.Generator(device="cuda")
    g.manual_seed(1)
    x = torch.randn(N, 3, 224, 224, device="cuda", generator=g)
    dp = torch.randn(N, 56, 56, 64, device="cuda", generator=g).to(torch.bfloat16)
    rm0 = bn.running_mean.clone()
    out, dw, dg, db, mean, var = _ref(conv, bn, x, dp)
    got = _run(conv, bn, pool, x, dp, fused=True)
    assert got.shape == (N, 56, 56, 64)
    assert _rel(got, out) < 2e-2
    # running statistics: momentum 0.1 update from the batch mean / unbiased variance
    assert _rel(bn.running_mean, 0.9 * rm0 + 0.1 * mean) < 1e-3
    cnt = N * 112 * 112
    assert _rel(bn.running_var, 0.9 + 0.1 * var * cnt / (cnt - 1)) < 1e-3
    assert _rel(conv.weight.grad, dw) < 3e-2
    assert _rel(bn.weight.grad, dg) < 3e-2
    assert _rel(bn.bias.grad, db) < 3e-2


def test_fused_stem_matches_unfused_kernels():
    conv, bn, pool = _stem(seed=3)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    g = torch.Generator(device="cuda")
    g.manual_seed(2)
    x = torch.randn(4, 3, 224, 224, device="cuda", generator=g)
    dp = torch.randn(4, 56, 56, 64, device="cuda", generator=g).to(torch.bfloat16)
    a = _run(conv, bn, pool, x, dp, fused=True)
    b = _run(conv2, bn2, pool, x, dp, fused=False)
    # the conv's fp32 sums differ only in order: rare 1-ulp bf16 differences in y
    assert (a.float() - b.float()).abs().max().item() < 0.05
    assert (a != b).float().mean().item() < 1e-2
    assert _rel(bn.running_mean, bn2.running_mean) < 1e-4
    assert _rel(bn.running_var, bn2.running_var) < 1e-4
    assert _rel(conv.weight.grad, conv2.weight.grad) < 1e-2
    assert _rel(bn.weight.grad, bn2.weight.grad) < 1e-2
    assert _rel(bn.bias.grad, bn2.bias.grad) < 1e-2


def test_fused_stem_deterministic_bitwise():
    set_deterministic(True)
    res = []
    for _ in range(2):
        conv, bn, pool = _stem(seed=4)
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        x = torch.randn(2, 3, 224, 224, device="cuda", generator=g)
        dp = torch.randn(2, 56, 56, 64, device="cuda", generator=g).to(torch.bfloat16)
        out = _run(conv, bn, pool, x, dp, fused=True)
        res.append((out, conv.weight.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone(),
                    bn.running_var.clone()))
    for u, v in zip(*res):
        assert torch.equal(u, v)


def test_fused_stem_eval_matches_unfused():
    conv, bn, pool = _stem(seed=6)
    with torch.no_grad():
        bn.running_var.uniform_(0.5, 2.0)
    conv.eval()
    bn.eval()
    x = torch.randn(2, 3, 224, 224, device="cuda")
    with torch.no_grad():
        xp = conv.pack_input(x, torch.bfloat16)
        MF.set_stem_fused(True)
        a = mnn.conv_bn_relu_maxpool(xp, conv, bn, pool)
        MF.set_stem_fused(False)
        b = mnn.conv_bn_relu_maxpool(xp, conv, bn, pool)
    assert (a.float() - b.float()).abs().max().item() < 0.05
    assert (a != b).float().mean().item() < 1e-2


def test_fused_stem_multi_band_blocks_match_unfused():
    """Enough images that the weight-grad blocks loop over several bands each (the half-band
    kernel runs min(N*56, 512) blocks)."""
    conv, bn, pool = _stem(seed=7)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    g = torch.Generator(device="cuda")
    g.manual_seed(8)
    x = torch.randn(24, 3, 224, 224, device="cuda", generator=g)
    dp = torch.randn(24, 56, 56, 64, device="cuda", generator=g).to(torch.bfloat16)
    _run(conv, bn, pool, x, dp, fused=True)
    _run(conv2, bn2, pool, x, dp, fused=False)
    assert _rel(conv.weight.grad, conv2.weight.grad) < 1e-2
    assert _rel(bn.weight.grad, bn2.weight.grad) < 1e-2
    assert _rel(bn.bias.grad, bn2.bias.grad) < 1e-2


def test_fused_stem_small_gamma_large_beta():
    """The fused backward recovers x̂ = (z-β)/γ from the bf16 pooled output, whose rounding error
    grows with |β/γ|; the unfused path takes x̂ from y.  Pinned here at |β/γ| up to 20 (init
    values are γ = 1, β = 0)."""
    conv, bn, pool = _stem(seed=9)
    with torch.no_grad():
        bn.weight.uniform_(0.05, 0.1)
        bn.bias.uniform_(0.5, 1.0)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    g = torch.Generator(device="cuda")
    g.manual_seed(10)
    x = torch.randn(4, 3, 224, 224, device="cuda", generator=g)
    dp = torch.randn(4, 56, 56, 64, device="cuda", generator=g).to(torch.bfloat16)
    _run(conv, bn, pool, x, dp, fused=True)
    _run(conv2, bn2, pool, x, dp, fused=False)
    e = [_rel(conv.weight.grad, conv2.weight.grad), _rel(bn.weight.grad, bn2.weight.grad),
         _rel(bn.bias.grad, bn2.bias.grad)]
    print("small-gamma stem: rel err dW, dgamma, dbeta vs unfused:", e)
    assert max(e) < 2e-2, e
