"""VGG / AlexNet on the mipipe op layer vs torchvision-structured plain-torch models (fp64),
torchvision state_dict key compatibility, and registry coverage of task.py's --arch families."""
import pytest
import torch

from mipipe.models import create_model, model_names
from mipipe.models.reference import RefAlexNet, RefVGG
from mipipe.ops.functional import cross_entropy


def test_registry_has_torchvision_families():
    names = set(model_names())
    for n in ["alexnet", "vgg11", "vgg11_bn", "vgg13", "vgg16", "vgg16_bn", "vgg19", "vgg19_bn",
              "resnet18", "resnet50", "wide_resnet50_2"]:
        assert n in names, n


@pytest.mark.parametrize("arch,res", [("vgg11", 32), ("vgg11_bn", 32), ("alexnet", 64)])
def test_fp64_parity(arch, res):
    torch.manual_seed(0)
    m = create_model(arch, num_classes=10, dropout=0.0).double()
    m.compute_dtype = torch.float64
    r = (RefAlexNet(num_classes=10, dropout=0.0) if arch == "alexnet"
         else RefVGG(arch, num_classes=10, dropout=0.0)).double()
    assert set(m.state_dict()) == set(r.state_dict())
    r.load_state_dict(m.state_dict())
    x = torch.randn(4, 3, res, res, dtype=torch.float64)
    y = torch.randint(0, 10, (4,))
    out, ref = m(x), r(x)
    assert (out - ref).abs().max() < 1e-9 * max(1.0, ref.abs().max().item())
    cross_entropy(out, y).backward()
    torch.nn.functional.cross_entropy(ref, y).backward()
    for (n, p), (_, q) in zip(m.named_parameters(), r.named_parameters()):
        assert (p.grad - q.grad).abs().max() <= 1e-7 * q.grad.abs().max() + 1e-12, n
