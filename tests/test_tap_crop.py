"""Filter-tap cropping (ops/functional.py::tap_crop): convolutions whose geometry never lets
some taps touch the image (3x3 / pad 1 on a 1x1 map; 3x3 / stride 2 / pad 1 on a 2x2 map — the
reference's ResNet-18 layer 4 at 32x32) run the smaller filter in the forward, data-grad and
weight-grad; results must equal the full filter (CPU float64 here, GPU kernels in
test_tap_crop_gpu below)."""
import pytest
import torch

from mipipe.ops import functional as MF


def test_tap_crop_geometry():
    assert MF.tap_crop((8, 1, 1, 512), (512, 3, 3, 512), 1, 1) == (1, 2, 1, 2, 0)
    assert MF.tap_crop((8, 2, 2, 256), (512, 3, 3, 256), 2, 1) == (1, 3, 1, 3, 0)
    assert MF.tap_crop((8, 2, 2, 256), (256, 3, 3, 256), 1, 1) is None  # every tap used
    assert MF.tap_crop((8, 7, 7, 512), (512, 3, 3, 512), 1, 1) is None
    assert MF.tap_crop((8, 1, 1, 64), (64, 3, 3, 64), (1, 1), 1) is None  # tuple stride: off
    assert MF.tap_crop((8, 1, 2, 64), (64, 3, 3, 64), 1, 1) is None  # non-square cropped pad


def _run(x, w, stride, pad, crop_on, dev, dtype):
    from mipipe import nn as mnn
    old = MF._TAP_CROP
    MF._TAP_CROP = crop_on
    try:
        conv = mnn.Conv2d(w.shape[1], w.shape[0], w.shape[2], stride=stride, padding=pad).to(dev)
        with torch.no_grad():
            conv.weight.copy_(w)
        conv.weight.data = conv.weight.data.to(dtype if dtype == torch.float64 else torch.float32)
        xi = x.clone().to(dev, dtype).requires_grad_(True)
        y = conv(xi)
        g = torch.randn(y.shape, generator=torch.Generator().manual_seed(1), dtype=torch.float64)
        (y.double() * g.to(dev)).sum().backward()
        return y.detach().double().cpu(), xi.grad.double().cpu(), conv.weight.grad.double().cpu()
    finally:
        MF._TAP_CROP = old


@pytest.mark.parametrize("H,stride,k,pad", [(1, 1, 3, 1), (2, 2, 3, 1), (3, 1, 3, 0), (2, 2, 2, 0)])
def test_cropped_conv_equals_full_filter_cpu(H, stride, k, pad):
    """(1,1,3,1): centre tap only; (2,2,3,1): 2x2 taps, then the flattened single-output
    form; (3,1,3,0) / (2,2,2,0): whole-image filters, flattened without a crop."""
    torch.manual_seed(0)
    x = torch.randn(4, H, H, 16, dtype=torch.float64)
    w = torch.randn(24, 16, k, k, dtype=torch.float64)
    full = _run(x, w, stride, pad, False, "cpu", torch.float64)
    crop = _run(x, w, stride, pad, True, "cpu", torch.float64)
    for a, b in zip(full, crop):
        assert torch.allclose(a, b, rtol=1e-12, atol=1e-12)
    # the cropped-away taps get exactly zero gradient
    if H == 1:
        assert float(crop[2][:, :, [0, 2], :].abs().max()) == 0.0


def test_flattened_conv_inside_resnet_block_cpu():
    """ResNet-18 at 32x32 runs layer 4's first conv flattened (its input is the previous block's
    fused BN+ReLU output): the module tree still matches the plain float64 reference (the
    per-channel BN-backward fusion is skipped for the flattened data-grad)."""
    from pinned_ref import pinned_grads
    from mipipe.models import create_model
    torch.manual_seed(0)
    m = create_model("resnet18", num_classes=10, compute_dtype=torch.float64).double()
    state = {kk: v.clone() for kk, v in m.state_dict().items()}
    names = [n for n, _ in m.named_parameters()]
    x = torch.randn(4, 3, 32, 32, dtype=torch.float64)
    y = torch.randint(0, 10, (4,))
    torch.nn.functional.cross_entropy(m(x), y).backward()
    _, _, g, _ = pinned_grads(state, names, x, y, None)
    for n, p in m.named_parameters():
        assert ((p.grad - g[n]).norm() / g[n].norm()).item() < 1e-10, n


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("H,stride,Ci,Co", [(1, 1, 512, 512), (2, 2, 256, 512)])
def test_tap_crop_gpu(dtype, H, stride, Ci, Co):
    """The GPU kernels on the cropped filter (1x1 / 2x2) == the full 3x3 filter through the
    implicit-GEMM kernels, forward / data-grad / weight-grad."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.manual_seed(0)
    x = torch.randn(64, H, H, Ci, dtype=torch.float64)
    w = torch.randn(Co, Ci, 3, 3, dtype=torch.float64) / (Ci * 9) ** 0.5
    full = _run(x, w, stride, 1, False, "cuda", dtype)
    crop = _run(x, w, stride, 1, True, "cuda", dtype)
    tol = 1e-4 if dtype == torch.float32 else 2e-2
    for a, b in zip(full, crop):
        err = ((a - b).abs().max() / (a.abs().max() + 1e-12)).item()
        assert err < tol, err
