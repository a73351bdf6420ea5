"""Model zoo on the CPU reference path: torchvision-compatible state_dict layout and exact
(fp64) parity of the fused conv/BN/residual autograd functions with plain torch.nn models."""
import pytest
import torch

from mipipe.models import create_model, model_names
from mipipe.models.reference import RefMnistCNN, ref_resnet

# torchvision resnet18 state_dict facts: 62 params + 60 buffers = 122 entries
TV_RESNET18_KEYS = ["conv1.weight", "bn1.running_mean", "layer1.0.conv1.weight",
                    "layer2.0.downsample.0.weight", "layer2.0.downsample.1.num_batches_tracked",
                    "fc.bias"]


def test_registry():
    names = model_names()
    for n in ["resnet18", "resnet34", "resnet50", "resnet101", "resnet152", "mnist_cnn"]:
        assert n in names
    assert names == sorted(names)


def test_resnet18_state_dict_layout():
    m = create_model("resnet18")
    sd = m.state_dict()
    assert len(sd) == 122
    assert sum(1 for _ in m.parameters()) == 62
    for k in TV_RESNET18_KEYS:
        assert k in sd
    assert sum(p.numel() for p in m.parameters()) == 11689512
    assert sd["conv1.weight"].shape == (64, 3, 7, 7)
    assert sd["layer2.0.downsample.1.num_batches_tracked"].dtype == torch.int64
    assert m.conv1.weight.is_contiguous(memory_format=torch.channels_last)


def test_resnet50_param_count():
    m = create_model("resnet50")
    assert sum(p.numel() for p in m.parameters()) == 25557032
    assert sum(1 for _ in m.parameters()) == 161


@pytest.mark.parametrize("arch", ["resnet18", "resnet50", "mnist_cnn"])
def test_fp64_parity_with_reference(arch):
    torch.manual_seed(0)
    kw = {"num_classes": 10}
    m = create_model(arch, compute_dtype=torch.float64, **kw).double()
    r = (RefMnistCNN() if arch == "mnist_cnn" else ref_resnet(arch, num_classes=10)).double()
    r.load_state_dict(m.state_dict(), strict=True)
    x = torch.randn(4, 1, 28, 28, dtype=torch.float64) if arch == "mnist_cnn" else \
        torch.randn(4, 3, 32, 32, dtype=torch.float64)
    y, yr = m(x), r(x)
    assert (y - yr).abs().max() < 1e-9
    w = torch.randn_like(y)
    (y * w).sum().backward()
    (yr * w).sum().backward()
    for (n, p), (_, q) in zip(m.named_parameters(), r.named_parameters()):
        assert (p.grad - q.grad).abs().max() <= 1e-6 * (q.grad.abs().max() + 1e-12), n
    for (n, b), (_, c) in zip(m.named_buffers(), r.named_buffers()):
        assert torch.allclose(b.double(), c.double(), atol=1e-9), n
    m.eval()
    r.eval()
    assert (m(x) - r(x)).abs().max() < 1e-9


def test_eval_mode_bn_backward_matches():
    torch.manual_seed(1)
    m = create_model("resnet18", num_classes=10, compute_dtype=torch.float64).double().eval()
    r = ref_resnet("resnet18", num_classes=10).double().eval()
    r.load_state_dict(m.state_dict())
    x = torch.randn(2, 3, 32, 32, dtype=torch.float64)
    m(x).sum().backward()
    r(x).sum().backward()
    for (n, p), (_, q) in zip(m.named_parameters(), r.named_parameters()):
        assert (p.grad - q.grad).abs().max() <= 1e-9 * (q.grad.abs().max() + 1e-12), n
