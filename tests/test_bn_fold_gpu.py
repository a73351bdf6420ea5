"""Folded BatchNorm (nn.conv_bn_act(fold_next=)): the BN + ReLU apply of a ResNet Bottleneck's
conv2 output runs inside conv3 — its forward A fragments and its weight-grad B fragments are
transformed to relu(y*scale + bias) after the LDS read — instead of as a separate pass that
writes the normalised tensor.  The transform reproduces bn_act_fwd's stored bits, so every
check here is bit-exact against the unfolded path on the same tile plan."""
import pytest
import torch

from mipipe import nn as mnn
from mipipe.ops import _ref
from mipipe.ops import determinism
from mipipe.ops import kernels as K
from mipipe.ops._native import native, native_available

pytestmark = pytest.mark.gpu
dev = "cuda"


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_available()
    yield
    determinism.set_deterministic(False)


def _bn(C, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    scale = torch.rand(C, device=dev, generator=g) + 0.5
    bias = torch.randn(C, device=dev, generator=g) * 0.5
    return scale, bias


# N, H, W, Ci, Co: ResNet-50 conv3 shapes (scaled batch), odd pixel counts (a k-tail in the
# weight-grad: N*H*W % 64 != 0) and channel counts that are not multiples of 64
SHAPES = [(4, 14, 14, 64, 256), (2, 7, 7, 512, 2048), (3, 5, 7, 40, 72), (1, 9, 9, 128, 24)]


@pytest.mark.parametrize("tile", list(range(11)))
@pytest.mark.parametrize("shape", SHAPES)
def test_folded_bn_forward_and_wgrad_bit_exact(tile, shape):
    N, H, W, Ci, Co = shape
    torch.manual_seed(tile)
    y = torch.randn(N, H, W, Ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, 1, 1, Ci, device=dev) / Ci ** 0.5).to(torch.bfloat16)
    scale, bias = _bn(Ci, 1)
    shift = torch.randn(Co, device=dev) * 0.1
    z = K.bn_act_fwd(y, scale, bias, True)  # the tensor the fold never writes
    # (torch's separate multiply and add round twice; the kernels' fused multiply-add once)
    assert torch.allclose(z.float(), _ref.bn_relu_fold(y, scale, bias).float(), rtol=1e-2,
                          atol=1e-2)
    ref = native().conv_fwd(z, w, 1, 0, shift, cfg=tile)
    got = native().conv_fwd(y, w, 1, 0, shift, cfg=tile, in_scale=scale, in_bias=bias)
    assert torch.equal(got[0], ref[0])
    assert torch.allclose(got[1].sum(0), ref[1].sum(0), rtol=1e-5, atol=1e-4)
    dy = torch.randn(N, H, W, Co, device=dev).to(torch.bfloat16)
    for sp in (1, 0, 3):  # unsplit read-modify-write, heuristic split-K, 3-way split-K
        cfg = tile + 16 * sp
        a = native().conv_wgrad(dy, z, 1, 1, 1, 0, cfg=cfg)
        b = native().conv_wgrad(dy, y, 1, 1, 1, 0, cfg=cfg, in_scale=scale, in_bias=bias)
        if sp == 1:
            assert torch.equal(a, b), (a - b).abs().max()
        else:  # fp32 atomics: order-dependent rounding only
            assert torch.allclose(a, b, rtol=1e-4, atol=1e-4), (a - b).abs().max()
    with determinism.deterministic(True):
        a = native().conv_wgrad(dy, z, 1, 1, 1, 0, cfg=tile + 16 * 3)
        b = native().conv_wgrad(dy, y, 1, 1, 1, 0, cfg=tile + 16 * 3, in_scale=scale,
                                in_bias=bias)
        assert torch.equal(a, b)


def test_folded_bn_rejects_unsupported_shapes():
    y = torch.randn(2, 8, 8, 64, device=dev).to(torch.bfloat16)
    s, b = _bn(64, 2)
    w3 = torch.randn(64, 3, 3, 64, device=dev).to(torch.bfloat16)
    with pytest.raises(RuntimeError):
        native().conv_fwd(y, w3, 1, 1, None, in_scale=s, in_bias=b)
    with pytest.raises(RuntimeError):
        native().conv_fwd(y.float(), w3[:, :1, :1].float().contiguous(), 1, 0, None,
                          in_scale=s, in_bias=b)


def _bottleneck_step(fold, det, steps=2):
    from mipipe.models import create_model
    from mipipe.optim import SGD
    from mipipe.ops.functional import cross_entropy
    old = (mnn._BN_FOLD, mnn._BN_FOLD_MODE)
    mnn._BN_FOLD, mnn._BN_FOLD_MODE = fold, ("1" if fold else "0")  # every size (small model)
    try:
        with determinism.deterministic(det):
            torch.manual_seed(0)
            m = create_model("resnet50", num_classes=10).to(dev)
            opt = SGD(m.parameters(), 0.1, momentum=0.9, weight_decay=1e-4)
            g = torch.Generator(device=dev).manual_seed(5)
            x = torch.randn(8, 3, 64, 64, device=dev, generator=g)
            t = torch.randint(0, 10, (8,), device=dev, generator=g)
            losses = []
            for _ in range(steps):
                opt.zero_grad()
                loss = cross_entropy(m(x), t)
                loss.backward()
                opt.step()
                losses.append(loss.detach())
            torch.cuda.synchronize()
            grads = [p.grad.detach().clone() for p in m.parameters()]
            state = [v.detach().float().clone() for v in m.state_dict().values()]
            return torch.stack(losses), grads, state
    finally:
        mnn._BN_FOLD, mnn._BN_FOLD_MODE = old


def test_resnet50_step_folded_equals_unfolded_deterministic():
    """Two SGD steps of ResNet-50 (every Bottleneck's BN2 folded into conv3) in deterministic
    mode: losses, every gradient and every parameter / buffer bit-identical to the unfolded
    model (same heuristic tile plans, fixed-order reductions)."""
    la, ga, sa = _bottleneck_step(True, True)
    lb, gb, sb = _bottleneck_step(False, True)
    assert torch.equal(la, lb), (la, lb)
    for i, (a, b) in enumerate(zip(ga, gb)):
        assert torch.equal(a, b), (i, (a - b).abs().max())
    for a, b in zip(sa, sb):
        assert torch.equal(a, b)


def test_resnet50_step_folded_close_default_mode():
    """Default mode (fp32 atomics in the statistics and split-K: run-to-run rounding noise, which
    a random-init net at lr 0.1 amplifies over steps — so one step): same loss, gradients within
    the atomics-order noise of the unfolded model."""
    la, ga, _ = _bottleneck_step(True, False, steps=1)
    lb, gb, _ = _bottleneck_step(False, False, steps=1)
    assert torch.allclose(la, lb, rtol=1e-3, atol=1e-3), (la, lb)
    num = sum(float((a - b).norm() ** 2) for a, b in zip(ga, gb)) ** 0.5
    den = sum(float(b.norm() ** 2) for b in gb) ** 0.5
    assert num / den < 2e-2, num / den
