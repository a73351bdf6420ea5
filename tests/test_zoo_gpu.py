"""gfx950 kernels of vision.hip (grouped / depthwise / non-square direct conv, any-C BatchNorm,
k x k average pool, ceil-mode max pool) vs the fp32 PyTorch reference of the same contract, and
the torchvision zoo models (MobileNetV2, MNASNet, ShuffleNetV2, SqueezeNet, DenseNet, GoogLeNet,
Inception-v3, ResNeXt) training on the GPU through mipipe's kernels.
Run on an MI355X:  python -m pytest tests -m gpu
"""
import math

import pytest
import torch

from mipipe.ops import _ref
from mipipe.ops._native import native, native_available

pytestmark = pytest.mark.gpu
dev = "cuda"
ACT = {"none": 0, "relu": 1, "relu6": 2}


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_available(), "mipipe._C must be built for GPU tests (no silent fallback)"
    torch.manual_seed(1234)


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


GCONV_CASES = [
    # N, H, W, Ci, Co, (kh, kw), (sh, sw), (ph, pw), groups
    (2, 14, 14, 96, 96, (3, 3), (1, 1), (1, 1), 96),       # depthwise, 8-channel vector path
    (2, 15, 15, 144, 144, (3, 3), (2, 2), (1, 1), 144),    # depthwise, stride 2
    (2, 9, 9, 40, 40, (5, 5), (2, 2), (2, 2), 40),         # depthwise 5x5 (MNASNet)
    (2, 7, 7, 58, 58, (3, 3), (1, 1), (1, 1), 58),         # depthwise, C % 8 != 0 (ShuffleNet)
    (2, 8, 8, 128, 128, (3, 3), (2, 2), (1, 1), 32),       # ResNeXt 32x4d group conv
    (2, 9, 11, 64, 48, (1, 7), (1, 1), (0, 3), 1),         # Inception 1x7
    (2, 9, 11, 48, 64, (7, 1), (1, 1), (3, 0), 1),         # Inception 7x1
    (2, 10, 10, 24, 58, (1, 1), (1, 1), (0, 0), 1),        # odd Co (ShuffleNet x1.0)
]


@pytest.mark.parametrize("case", GCONV_CASES)
@pytest.mark.parametrize("act", ["none", "relu6"])
def test_gconv_fwd_dgrad_wgrad(case, act):
    N, H, W, Ci, Co, k, s, p, g = case
    x = bf(N, H, W, Ci)
    w = bf(Co, k[0], k[1], Ci // g, scale=1.0 / math.sqrt(Ci // g * k[0] * k[1]))
    b = torch.randn(Co, device=dev) * 0.1
    y = native().gconv_fwd(x, w, list(s), list(p), g, b, ACT[act])
    yr = _ref.gconv_fwd(x.float(), w.float(), s, p, g, b, act)
    assert y.shape == yr.shape
    assert rel_err(y, yr) < 1e-2
    dy = bf(*y.shape)
    z = y if act != "none" else None
    dx = native().gconv_dgrad(dy, w, [N, H, W, Ci], list(s), list(p), g, z, ACT[act])
    dxr = _ref.gconv_dgrad(dy.float(), w.float(), (N, H, W, Ci), s, p, g, z, act)
    assert rel_err(dx, dxr) < 1e-2
    dw, db = native().gconv_wgrad(dy, x, k[0], k[1], list(s), list(p), g, z, ACT[act], None, None,
                                  True)
    dwr, dbr = _ref.gconv_wgrad(dy.float(), x.float(), k[0], k[1], s, p, g, z, act)
    assert rel_err(dw, dwr) < 1e-2
    assert rel_err(db, dbr) < 1e-2
    # accumulation into an existing buffer (the flat-gradient path)
    acc = torch.ones_like(dwr)
    native().gconv_wgrad(dy, x, k[0], k[1], list(s), list(p), g, z, ACT[act], acc)
    assert rel_err(acc - 1, dwr) < 1e-2


@pytest.mark.parametrize("k,p", [((1, 7), (0, 3)), ((7, 1), (3, 0)), ((1, 3), (0, 1)),
                                 ((3, 1), (1, 0))])
def test_mfma_conv_nonsquare_padding(k, p):
    """Inception-v3's 1xn / nx1 convs on the MFMA implicit-GEMM kernels (separate h / w
    padding): forward with the BN-statistics epilogue, dgrad, wgrad."""
    N, H, W, Ci, Co = 2, 17, 13, 64, 96
    x = bf(N, H, W, Ci)
    w = bf(Co, k[0], k[1], Ci, scale=1.0 / math.sqrt(Ci * k[0] * k[1]))
    shift = torch.randn(Co, device=dev) * 0.1
    y, ps, pss = native().conv_fwd(x, w, 1, p[0], shift, pad_w=p[1])
    yr, psr, pssr = _ref.conv_fwd(x.float(), w.float(), 1, p, shift)
    assert y.shape == yr.shape and rel_err(y, yr) < 1e-2
    assert rel_err(ps.sum(0), psr[0]) < 2e-3 and rel_err(pss.sum(0), pssr[0]) < 2e-3
    dy = bf(*y.shape)
    dx = native().conv_dgrad(dy, w, [N, H, W, Ci], 1, p[0], pad_w=p[1])
    assert rel_err(dx, _ref.conv_dgrad(dy.float(), w.float(), (N, H, W, Ci), 1, p)) < 1e-2
    dw = native().conv_wgrad(dy, x, k[0], k[1], 1, p[0], pad_w=p[1])
    assert rel_err(dw, _ref.conv_wgrad(dy.float(), x.float(), k[0], k[1], 1, p)) < 1e-2


@pytest.mark.parametrize("Ci,groups,stride", [(128, 32, 1), (256, 32, 2), (512, 32, 1),
                                              (2048, 32, 1)])
def test_block_group_conv_mfma(Ci, groups, stride):
    """ResNeXt grouped 3x3 convs as block-diagonal dense convs on the MFMA kernels, vs torch's
    fp32 grouped conv (forward, input and weight gradients through autograd)."""
    from mipipe.ops import functional as MF
    N, H = 2, 9
    cig = Ci // groups
    gb = MF.grouped_conv_mfma_blocks(groups, cig, cig)
    assert gb > 0
    x = bf(N, H, H, Ci).requires_grad_()
    wp = (torch.randn(Ci, cig, 3, 3, device=dev) / math.sqrt(cig * 9)).requires_grad_()
    w_c = wp.detach().permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    y = MF.block_group_conv2d(x, wp, w_c, stride, 1, groups, gb)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    wr = w_c.float().permute(0, 3, 1, 2).detach().requires_grad_()
    yr = torch.nn.functional.conv2d(xr, wr, stride=stride, padding=1, groups=groups)
    assert rel_err(y, yr.permute(0, 2, 3, 1)) < 1e-2
    dy = bf(*y.shape)
    y.backward(dy)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert rel_err(x.grad, xr.grad.permute(0, 2, 3, 1)) < 1e-2
    assert rel_err(wp.grad, wr.grad) < 1e-2


@pytest.mark.parametrize("C", [58, 96, 24, 200])
@pytest.mark.parametrize("act", ["none", "relu", "relu6"])
def test_bn_generic(C, act):
    y = bf(3, 7, 9, C, scale=2.0) + 0.5
    shift = torch.randn(C, device=dev) * 0.1
    ps, pq = native().chan_stats(y, shift)
    assert ps.shape[0] == native().STAT_REPLICAS  # replica rows, summed by bn_finalize
    psr, pqr = _ref.chan_stats(y.float(), shift)
    ps, pq = ps.sum(0).reshape(psr.shape), pq.sum(0).reshape(pqr.shape)
    assert rel_err(ps, psr) < 1e-3 and rel_err(pq, pqr) < 1e-3
    scale, bias = torch.randn(C, device=dev), torch.randn(C, device=dev)
    z = native().affine_act(y, scale, bias, ACT[act])
    assert rel_err(z, _ref.affine_act(y.float(), scale, bias, act)) < 1e-2
    mean, invstd = torch.randn(C, device=dev) * 0.1, torch.rand(C, device=dev) + 0.5
    gamma = torch.randn(C, device=dev)
    dz = bf(*y.shape)
    zz = z if act != "none" else None
    sg, sgx = native().bn_generic_bwd_reduce(dz, zz, y, mean, invstd, ACT[act])
    sgr, sgxr = _ref.bn_generic_bwd_reduce(dz.float(), zz, y.float(), mean, invstd, act)
    assert rel_err(sg, sgr) < 1e-3 and rel_err(sgx, sgxr) < 1e-3
    count = y.numel() // C
    dy = native().bn_generic_bwd_apply(dz, zz, y, mean, invstd, gamma, sg, sgx, count, ACT[act])
    dyr = _ref.bn_generic_bwd_apply(dz.float(), zz, y.float(), mean, invstd, gamma, sgr, sgxr,
                                    count, act)
    assert rel_err(dy, dyr) < 1e-2
    dye = native().bn_generic_bwd_apply(dz, zz, y, mean, invstd, gamma, None, None, count, ACT[act])
    assert rel_err(dye, _ref.bn_generic_bwd_apply(dz.float(), zz, y.float(), mean, invstd, gamma,
                                                  None, None, count, act)) < 1e-2


@pytest.mark.parametrize("k,s,p", [(2, 2, 0), (3, 1, 1), (5, 3, 0)])
@pytest.mark.parametrize("C", [64, 58])
def test_avgpool2d(k, s, p, C):
    x = bf(2, 17, 17, C)
    y = native().avgpool2d_fwd(x, k, s, p)
    yr = _ref.avgpool2d_fwd(x.float(), k, s, p)
    assert y.shape == yr.shape and rel_err(y, yr) < 1e-2
    dy = bf(*y.shape)
    dx = native().avgpool2d_bwd(dy, list(x.shape), k, s, p)
    assert rel_err(dx, _ref.avgpool2d_bwd(dy.float(), tuple(x.shape), k, s, p)) < 1e-2


@pytest.mark.parametrize("H,k,s,p", [(13, 3, 2, 0), (14, 3, 2, 0), (7, 3, 1, 1), (9, 2, 2, 0)])
def test_maxpool_ceil_mode(H, k, s, p):
    x = bf(2, H, H, 64)
    y, idx = native().maxpool_fwd(x, k, s, p, True)
    ref = torch.nn.functional.max_pool2d(x.float().permute(0, 3, 1, 2), k, s, p, ceil_mode=True)
    assert y.shape == ref.permute(0, 2, 3, 1).shape
    assert torch.equal(y.float(), ref.permute(0, 2, 3, 1))
    dy = bf(*y.shape)
    dx = native().maxpool_bwd_impl(dy, idx, list(x.shape), k, s, p)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    torch.nn.functional.max_pool2d(xr, k, s, p, ceil_mode=True).backward(dy.float().permute(0, 3, 1, 2))
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


ZOO = [("mobilenet_v2", 64), ("mnasnet1_0", 64), ("shufflenet_v2_x1_0", 64),
       ("squeezenet1_1", 64), ("densenet121", 64), ("googlenet", 64), ("inception_v3", 299),
       ("resnext50_32x4d", 64)]
NODROP = {"mobilenet_v2": dict(dropout=0.0), "mnasnet1_0": dict(dropout=0.0),
          "squeezenet1_1": dict(dropout=0.0), "googlenet": dict(dropout=0.0, dropout_aux=0.0),
          "inception_v3": dict(dropout=0.0)}


def cos(a, b):
    """Scale-invariant cosine (eval-mode outputs of a random-init net can be ~1e-10)."""
    a, b = a.flatten().double(), b.flatten().double()
    a, b = a / (a.abs().max() + 1e-300), b / (b.abs().max() + 1e-300)
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


@pytest.mark.parametrize("arch,res", ZOO)
def test_zoo_eval_matches_fp32_torch(arch, res):
    """bf16 NHWC execution on mipipe's kernels vs the same weights run by fp32 torch (NCHW)."""
    from mipipe.models import create_model
    from mipipe.models.reference import ref_resnet
    torch.manual_seed(0)
    m = create_model(arch, num_classes=100, **NODROP.get(arch, {})).cuda().eval()
    x = torch.randn(4, 3, res, res, device=dev)
    if arch.startswith("resnext"):
        r = ref_resnet(arch, num_classes=100).cuda().eval()
        r.load_state_dict(m.state_dict())
        ref_fwd = r
    else:
        ref_fwd = m.reference_forward
    with torch.no_grad():
        out, ref = m(x), ref_fwd(x)
    assert cos(out, ref) > 0.99, cos(out, ref)


@pytest.mark.parametrize("arch,res", ZOO)
def test_zoo_train_steps_reduce_loss(arch, res):
    """A few SGD steps on one batch through the kernels (flat-buffer optimizer, fused grads)."""
    from mipipe.models import create_model
    from mipipe.optim import SGD
    from mipipe.train.task import CrossEntropyLoss
    torch.manual_seed(0)
    m = create_model(arch, num_classes=10).cuda()
    m.compute_dtype = torch.bfloat16
    opt = SGD(m.parameters(), 0.005, momentum=0.9, weight_decay=1e-4, shadow_dtype=torch.bfloat16)
    crit = CrossEntropyLoss()
    x = torch.randn(8, 3, res, res, device=dev)
    y = torch.randint(0, 10, (8,), device=dev)
    losses = []
    m.train()
    for _ in range(5):
        opt.zero_grad()
        loss = crit(m(x), y)
        loss.backward()
        opt.step()
        losses.append(float(loss.item()))
    assert all(math.isfinite(v) for v in losses), losses
    assert min(losses[1:]) < losses[0], losses
