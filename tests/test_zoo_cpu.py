"""The torchvision model zoo beyond ResNet / VGG, reachable through task.py's ``--arch`` registry
scan (reference task.py:50-52, 63-67, 166-171): MobileNetV2, MNASNet, ShuffleNetV2, SqueezeNet,
DenseNet, GoogLeNet, Inception-v3 and ResNeXt.

* layout: parameter counts equal torchvision's published figures (1000 classes) and keys follow
  torchvision's module tree, so checkpoints interchange;
* fp64 parity on the CPU path: mipipe's NHWC executor (``model(x)``: fused conv/BN/act units,
  grouped / depthwise / non-square convs, any-C BatchNorm, pooling) against the SAME module tree
  run by plain torch on NCHW (``model.reference_forward``) — outputs (incl. auxiliary heads),
  every parameter gradient, BN running statistics, and eval mode.
"""
import copy

import pytest
import torch

from mipipe.models import create_model, model_names
from mipipe.models.reference import ref_resnet
from mipipe.train.task import CrossEntropyLoss

# torchvision parameter counts (1000 classes; googlenet with its default aux heads)
TV_PARAMS = {
    "mobilenet_v2": 3504872, "mnasnet0_5": 2218512, "mnasnet0_75": 3170208,
    "mnasnet1_0": 4383312, "mnasnet1_3": 6282256,
    "shufflenet_v2_x0_5": 1366792, "shufflenet_v2_x1_0": 2278604,
    "shufflenet_v2_x1_5": 3503624, "shufflenet_v2_x2_0": 7393996,
    "squeezenet1_0": 1248424, "squeezenet1_1": 1235496,
    "densenet121": 7978856, "densenet161": 28681000, "densenet169": 14149480,
    "densenet201": 20013928, "resnext50_32x4d": 25028904, "resnext101_32x8d": 88791336,
    "googlenet": 13004888, "inception_v3": 27161264,
}

TV_KEYS = {
    "mobilenet_v2": ["features.0.0.weight", "features.1.conv.0.0.weight",
                     "features.1.conv.1.weight", "features.2.conv.0.0.weight",
                     "features.18.1.running_var", "classifier.1.bias"],
    "mnasnet1_0": ["layers.0.weight", "layers.8.0.layers.3.weight", "layers.14.weight",
                   "layers.15.num_batches_tracked", "classifier.1.weight"],
    "shufflenet_v2_x1_0": ["conv1.0.weight", "stage2.0.branch1.0.weight",
                           "stage2.1.branch2.3.weight", "conv5.1.running_mean", "fc.weight"],
    "squeezenet1_0": ["features.0.weight", "features.3.squeeze.weight",
                      "features.3.expand3x3.bias", "classifier.1.weight"],
    "densenet121": ["features.conv0.weight", "features.denseblock1.denselayer1.norm1.weight",
                    "features.denseblock1.denselayer1.conv2.weight",
                    "features.transition1.conv.weight", "features.norm5.running_mean",
                    "classifier.weight"],
    "googlenet": ["conv1.conv.weight", "conv1.bn.running_mean", "inception3a.branch2.1.conv.weight",
                  "inception3a.branch4.1.bn.weight", "aux1.fc1.weight", "aux2.conv.conv.weight",
                  "fc.weight"],
    "inception_v3": ["Conv2d_1a_3x3.conv.weight", "Mixed_5b.branch5x5_2.conv.weight",
                     "Mixed_6b.branch7x7dbl_5.bn.running_var", "Mixed_7c.branch3x3dbl_3b.conv.weight",
                     "AuxLogits.conv1.conv.weight", "AuxLogits.fc.weight", "fc.bias"],
    "resnext50_32x4d": ["layer1.0.conv2.weight", "layer4.2.bn3.weight", "fc.weight"],
}


def test_registry_covers_torchvision():
    names = set(model_names())
    for n in TV_PARAMS:
        assert n in names, n


@pytest.mark.parametrize("arch", sorted(TV_PARAMS))
def test_param_count_matches_torchvision(arch):
    m = create_model(arch)
    assert sum(p.numel() for p in m.parameters()) == TV_PARAMS[arch]


def test_googlenet_without_aux_param_count():
    assert sum(p.numel() for p in create_model("googlenet", aux_logits=False).parameters()) == 6624904


@pytest.mark.parametrize("arch", sorted(TV_KEYS))
def test_state_dict_keys(arch):
    sd = create_model(arch).state_dict()
    for k in TV_KEYS[arch]:
        assert k in sd, (arch, k)
    shapes = {"resnext50_32x4d": ("layer1.0.conv2.weight", (128, 4, 3, 3)),
              "mobilenet_v2": ("features.1.conv.0.0.weight", (32, 1, 3, 3)),
              "inception_v3": ("Mixed_6b.branch7x7_2.conv.weight", (128, 128, 1, 7))}
    if arch in shapes:
        k, shp = shapes[arch]
        assert tuple(sd[k].shape) == shp


def _outs(o):
    return [t for t in (o if isinstance(o, tuple) else (o,)) if t is not None]


PARITY = [
    ("mobilenet_v2", dict(dropout=0.0), 32),
    ("mnasnet0_5", dict(dropout=0.0), 32),
    ("shufflenet_v2_x0_5", {}, 32),
    ("shufflenet_v2_x1_0", {}, 32),   # 58-channel branches: any-C conv / BN kernels
    ("squeezenet1_0", dict(dropout=0.0), 48),
    ("squeezenet1_1", dict(dropout=0.0), 48),
    ("densenet121", {}, 32),
    ("googlenet", dict(dropout=0.0, dropout_aux=0.0), 64),
    ("inception_v3", dict(dropout=0.0), 299),
    ("resnext50_32x4d", {}, 64),
]


@pytest.mark.parametrize("arch,kw,res", PARITY)
def test_fp64_parity_with_torch(arch, kw, res):
    torch.manual_seed(0)
    m = create_model(arch, num_classes=10, compute_dtype=torch.float64, **kw).double()
    if arch.startswith("resnext"):
        r = ref_resnet(arch, num_classes=10).double()
        r.load_state_dict(m.state_dict())
        ref_fwd = r.forward
    else:
        r = copy.deepcopy(m)
        ref_fwd = r.reference_forward
    x = torch.randn(2, 3, res, res, dtype=torch.float64)
    out, ref = _outs(m(x)), _outs(ref_fwd(x))
    assert len(out) == len(ref) == (3 if arch == "googlenet" else 2 if arch == "inception_v3" else 1)
    for a, b in zip(out, ref):
        assert (a - b).abs().max() <= 1e-7 * max(1.0, b.abs().max().item())
    ws = [torch.randn_like(a) for a in out]
    sum((a * w).sum() for a, w in zip(out, ws)).backward()
    sum((b * w).sum() for b, w in zip(ref, ws)).backward()
    # BN biases feeding conv->BN have an exactly-zero true gradient: compare against the global
    # gradient scale, not per tensor
    scale = max(q.grad.abs().max().item() for q in r.parameters())
    for (n, p), (_, q) in zip(m.named_parameters(), r.named_parameters()):
        assert p.grad is not None, n
        assert (p.grad - q.grad).abs().max() <= 1e-6 * scale, n
    for (n, b), (_, c) in zip(m.named_buffers(), r.named_buffers()):
        assert torch.allclose(b.double(), c.double(), rtol=1e-7, atol=1e-9), n
    m.eval()
    r.eval()
    a, b = m(x), ref_fwd(x)
    assert (a - b).abs().max() <= 1e-7 * max(1.0, b.abs().max().item())


def test_aux_logits_loss():
    """Training-mode GoogLeNet/Inception named tuples: main loss + weighted auxiliary losses."""
    from mipipe.models.inception import GoogLeNetOutputs, InceptionOutputs
    torch.manual_seed(0)
    y = torch.randint(0, 5, (4,))
    a, b, c = (torch.randn(4, 5) for _ in range(3))
    ce = CrossEntropyLoss()
    f = torch.nn.functional.cross_entropy
    assert torch.allclose(ce(GoogLeNetOutputs(a, b, c), y), f(a, y) + 0.3 * (f(b, y) + f(c, y)))
    assert torch.allclose(ce(InceptionOutputs(a, b), y), f(a, y) + 0.4 * f(b, y))
    assert torch.allclose(ce(a, y), f(a, y))


def test_task_trains_googlenet_on_cpu(tmp_path, monkeypatch):
    """task.py end to end with an aux-head architecture (the reference crashes on this)."""
    import json
    from mipipe.train import task as T
    monkeypatch.setenv("MIPIPE_FORCE_CPU", "1")
    monkeypatch.delenv("AIP_MODEL_DIR", raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    args = ["--arch", "googlenet", "--dataset", "cifar10", "--batch_size", "8",
            "--train-samples", "16", "--test-samples", "8", "--num_classes", "10",
            "--local_training", "--model_dir", str(tmp_path / "out"), "--num_epochs", "1",
            "--log-every", "0", "--metrics-file", str(tmp_path / "m.json")]
    assert T.main(args) == 0
    assert json.loads((tmp_path / "m.json").read_text())["steps"] == 2
