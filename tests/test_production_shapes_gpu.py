"""Every distinct ResNet-50 @224, batch-256 layer shape (the headline benchmark's config) through the
HIP kernels vs a plain-PyTorch fp32 evaluation of the same op on the same bf16-quantised inputs:
conv fwd (+BN statistics) / dgrad / wgrad (weight-grad reductions up to K = 256*56*56 = 802,816
pixels), the stem super-pixel conv, 3x3/2 max-pool on 256x112x112x64, BatchNorm on 2048
channels, the 2048->1000 classifier GEMMs and cross-entropy.  Bounds are bf16 output rounding
(1e-2 relative to the output magnitude; 5e-3 for fp32-accumulated reductions)."""
import math
import os
import sys

import pytest
import torch

from mipipe.ops import _ref
from mipipe.ops._native import native, native_available

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_kernels import resnet50_convs  # noqa: E402

pytestmark = pytest.mark.gpu
dev = "cuda"
B = 256


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_available()
    torch.manual_seed(11)
    yield
    torch.cuda.empty_cache()


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


SHAPES = [s for s in resnet50_convs(B) if s[0] != "stem"]


@pytest.mark.parametrize("shape", SHAPES, ids=[s[0] for s in SHAPES])
def test_resnet50_b256_conv_layer(shape):
    name, N, H, W, Ci, Co, k, s, p, _ = shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = bf(N, H, W, Ci)
    w = bf(Co, k, k, Ci, scale=1.0 / math.sqrt(Ci * k * k))
    shift = torch.randn(Co, device=dev) * 0.1
    y, ps, pss = native().conv_fwd(x, w, s, p, shift)
    yr, psr, pssr = _ref.conv_fwd(x.float(), w.float(), s, p, shift)
    assert rel(y, yr) < 1e-2
    assert rel(ps.sum(0), psr[0]) < 5e-3 and rel(pss.sum(0), pssr[0]) < 5e-3
    del y, yr
    dy = bf(N, Ho, Wo, Co)
    dx = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p)
    assert rel(dx, _ref.conv_dgrad(dy.float(), w.float(), (N, H, W, Ci), s, p)) < 1e-2
    del dx
    dw = native().conv_wgrad(dy, x, k, k, s, p)
    assert rel(dw, _ref.conv_wgrad(dy.float(), x.float(), k, k, s, p)) < 5e-3


def test_resnet50_b256_stem_maxpool_bn_head():
    from mipipe.models.resnet import _StemConv
    img = torch.randn(B, 3, 224, 224, device=dev)
    stem = _StemConv(3, 64, 7, stride=2, padding=3).to(dev)
    xp = stem.pack_input(img, torch.bfloat16)
    y, _, _ = native().conv_fwd(xp, stem.compute_weight(torch.bfloat16), 2, 0, None, stride_w=1)
    ref = torch.nn.functional.conv2d(img.to(torch.bfloat16).float(),
                                     stem.weight.detach().to(torch.bfloat16).float(), stride=2,
                                     padding=3).permute(0, 2, 3, 1)
    assert y.shape == (B, 112, 112, 64) and rel(y, ref) < 1e-2
    # 3x3/2 max-pool on the stem output, fwd + bwd
    mp, idx = native().maxpool_fwd(y, 3, 2, 1)
    mpr, _ = _ref.maxpool_fwd(y.float(), 3, 2, 1)
    assert torch.equal(mp.float(), mpr.float())
    g = bf(*mp.shape)
    dx = native().maxpool_bwd_impl(g, idx, list(y.shape), 3, 2, 1)
    yr = y.float().permute(0, 3, 1, 2).requires_grad_(True)
    torch.nn.functional.max_pool2d(yr, 3, 2, 1).backward(g.float().permute(0, 3, 1, 2))
    assert rel(dx, yr.grad.permute(0, 2, 3, 1)) < 1e-2
    # BatchNorm on 2048 channels (layer4 output, M = 256*7*7)
    C, M = 2048, B * 7 * 7
    yb = bf(M, C, scale=2.0)
    mean = yb.float().mean(0)
    var = yb.float().var(0, unbiased=False)
    invstd = torch.rsqrt(var + 1e-5)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev) * 0.1
    scale = gamma * invstd
    bias = beta - mean * scale
    z = native().bn_act_fwd(yb, scale, bias, True, None, None, None)
    zr = _ref.bn_act_fwd(yb.float(), scale, bias, True)
    assert rel(z, zr) < 1e-2
    dz = bf(M, C)
    sg, sgx, _ = native().bn_act_bwd_reduce(dz, z, yb, mean, invstd, True)
    sgr, sgxr = _ref.bn_act_bwd_reduce(dz.float(), z.float(), yb.float(), mean, invstd, True)
    assert rel(sg, sgr) < 5e-3 and rel(sgx, sgxr) < 5e-3
    # classifier: 2048 -> 1000 GEMMs + cross-entropy on 256 rows
    feat = bf(B, 2048)
    wfc = bf(1000, 2048, scale=0.02)
    bfc = torch.randn(1000, device=dev) * 0.01
    logits = native().gemm(feat, wfc, False, True, bfc, "none", torch.bfloat16, None, 0.0)
    assert rel(logits, _ref.gemm(feat.float(), wfc.float(), False, True, bfc, "none",
                                 torch.float32)) < 1e-2
    labels = torch.randint(0, 1000, (B,), device=dev)
    loss, grad = native().cross_entropy_fwd_bwd(logits, labels, 0.0, -100)
    lr_, gr = _ref.cross_entropy_fwd_bwd(logits.float(), labels)
    assert abs(loss.item() - lr_.item()) < 1e-3 * lr_.item() and rel(grad, gr) < 1e-2
    dwfc = native().gemm(grad, feat, True, False, None, "none", torch.float32, None, 0.0)
    assert rel(dwfc, grad.float().t() @ feat.float()) < 5e-3
