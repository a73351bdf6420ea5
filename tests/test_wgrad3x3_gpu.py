"""Patch-resident 3x3 weight-gradient kernel (csrc/kernels/wgrad3x3.hip) against the fp32
PyTorch reference (torch.nn.grad.conv2d_weight on the same bf16 operands).

Covers every ResNet-50 stride-1 3x3 layer shape class (k-step = 1 / 2 / 4 / 7 output rows of one
image, partial last row groups), odd spatial sizes, accumulation into an existing gradient (the
flat DDP bucket view), determinism, and agreement with the generic implicit-GEMM weight-grad."""
import pytest
import torch

from mipipe.ops import _ref
from mipipe.ops._native import native, native_available

pytestmark = pytest.mark.gpu

SHAPES = [  # N, H, W, Ci, Co
    (4, 56, 56, 64, 64),     # layer1: one row (56 px) per k-step
    (4, 28, 28, 128, 128),   # layer2: two rows
    (4, 14, 14, 256, 256),   # layer3: four rows, last group of an image has two
    (8, 7, 7, 512, 512),     # layer4: the whole 7x7 image per k-step
    (3, 9, 11, 64, 128),     # odd sizes, Co != Ci
    (2, 5, 30, 128, 64),
]


@pytest.fixture(autouse=True)
def _native():
    assert native_available()
    yield
    native().set_wgrad3x3(True)


def _data(N, H, W, Ci, Co, seed=0):
    g = torch.Generator(device="cuda")
    g.manual_seed(seed)
    x = torch.randn(N, H, W, Ci, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(N, H, W, Co, device="cuda", generator=g).to(torch.bfloat16)
    return x, dy


@pytest.mark.parametrize("shape", SHAPES, ids=[str(s) for s in SHAPES])
def test_wgrad3x3_matches_fp32_reference(shape):
    N, H, W, Ci, Co = shape
    x, dy = _data(*shape)
    ref = _ref.conv_wgrad(dy.float(), x.float(), 3, 3, 1, 1)
    native().set_wgrad3x3(True)
    out = native().conv_wgrad(dy, x, 3, 3, 1, 1)
    torch.cuda.synchronize()
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    assert err < 1e-4, err
    # accumulate into an existing gradient (flat-bucket view semantics)
    base = torch.randn_like(ref)
    acc = base.clone()
    native().conv_wgrad(dy, x, 3, 3, 1, 1, out=acc)
    err = ((acc - (base + ref)).abs().max() / ref.abs().max()).item()
    assert err < 1e-4, err
    # fixed-order partial sums: bit-reproducible
    again = native().conv_wgrad(dy, x, 3, 3, 1, 1)
    assert torch.equal(out, again)
    # and the generic implicit-GEMM weight-grad agrees
    native().set_wgrad3x3(False)
    gen = native().conv_wgrad(dy, x, 3, 3, 1, 1)
    native().set_wgrad3x3(True)
    err = ((gen - out).abs().max() / ref.abs().max()).item()
    assert err < 1e-4, err
