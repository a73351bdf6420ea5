"""Model zoo + registry with torchvision-style ``--arch`` semantics (task.py:50-52, 63-67).

``model_names()`` lists the lower-case constructor names, like the reference's scan of
``torchvision.models.__dict__``; ``create_model(arch, **kw)`` builds one.
"""
from __future__ import annotations

import glob
import os
from typing import Callable, Dict, List, Optional

from .resnet import (resnet18, resnet34, resnet50, resnet101, resnet152,  # noqa: F401
                     wide_resnet50_2, wide_resnet101_2, resnext50_32x4d, resnext101_32x8d,
                     ResNet)
from .cnn import mnist_cnn, MnistCNN  # noqa: F401

_REGISTRY: Dict[str, Callable] = {
    "resnet18": resnet18, "resnet34": resnet34, "resnet50": resnet50,
    "resnet101": resnet101, "resnet152": resnet152,
    "wide_resnet50_2": wide_resnet50_2, "wide_resnet101_2": wide_resnet101_2,
    "resnext50_32x4d": resnext50_32x4d, "resnext101_32x8d": resnext101_32x8d,
    "mnist_cnn": mnist_cnn,
}


def register_model(name: str, fn: Callable) -> None:
    _REGISTRY[name] = fn


_ZOO_MODULES = ("vgg", "mobilenet", "shufflenet", "squeezenet", "densenet", "inception", "bert")


def _lazy_register():
    """Import the remaining families (torchvision's registry: VGG/AlexNet, MobileNetV2, MNASNet,
    ShuffleNetV2, SqueezeNet, DenseNet, GoogLeNet, Inception-v3; plus BERT)."""
    import importlib
    for name in _ZOO_MODULES:
        importlib.import_module(f"{__name__}.{name}")


def model_names() -> List[str]:
    _lazy_register()
    return sorted(n for n in _REGISTRY if n.islower() and not n.startswith("__"))


def create_model(arch: str, **kw):
    _lazy_register()
    if arch not in _REGISTRY:
        raise KeyError(f"unknown arch {arch!r}; choices: {model_names()}")
    return _REGISTRY[arch](**kw)


def find_pretrained(arch: str, path: Optional[str] = None) -> Optional[str]:
    """Locate a torchvision-format weights file for ``arch`` without network access: ``path``
    when given, else torchvision's download cache ``$TORCH_HOME/hub/checkpoints/<arch>-*.pth``
    (``~/.cache/torch`` by default) — where ``models.<arch>(pretrained=True)`` (reference
    task.py:166-168) would have put it."""
    if path:
        return path if os.path.exists(path) else None
    home = os.environ.get("TORCH_HOME", os.path.join(os.path.expanduser("~"), ".cache", "torch"))
    ckpt = os.path.join(home, "hub", "checkpoints")
    # ``pretrained=True`` in torchvision 0.8 (the reference's container, nb:137) means the
    # IMAGENET1K_V1 weights: prefer that exact file when the cache holds several versions
    v1 = _TV_V1_FILES.get(arch)
    if v1 and os.path.exists(os.path.join(ckpt, v1)):
        return os.path.join(ckpt, v1)
    stem = _TV_V1_FILES.get(arch, f"{arch}-").split("-")[0]
    hits = sorted(set(glob.glob(os.path.join(ckpt, f"{arch}-*.pth")) +
                      glob.glob(os.path.join(ckpt, f"{stem}-*.pth"))))
    if len(hits) > 1:
        import warnings
        warnings.warn(f"find_pretrained({arch!r}): several weight files {hits}; none is the "
                      f"IMAGENET1K_V1 file {v1!r} the reference would load — using {hits[0]}")
    return hits[0] if hits else None


# torchvision's IMAGENET1K_V1 weight file names (what models.<arch>(pretrained=True) downloads)
_TV_V1_FILES = {
    "resnet18": "resnet18-f37072fd.pth", "resnet34": "resnet34-b627a593.pth",
    "resnet50": "resnet50-0676ba61.pth", "resnet101": "resnet101-63fe2227.pth",
    "resnet152": "resnet152-394f9c45.pth", "resnext50_32x4d": "resnext50_32x4d-7cdf4587.pth",
    "resnext101_32x8d": "resnext101_32x8d-8ba56ff5.pth",
    "wide_resnet50_2": "wide_resnet50_2-95faca4d.pth", "wide_resnet101_2": "wide_resnet101_2-32ee1156.pth",
    "alexnet": "alexnet-owt-7be5be79.pth", "vgg11": "vgg11-8a719046.pth", "vgg13": "vgg13-19584684.pth",
    "vgg16": "vgg16-397923af.pth", "vgg19": "vgg19-dcbb9e9d.pth", "vgg11_bn": "vgg11_bn-6002323d.pth",
    "vgg13_bn": "vgg13_bn-abd245e5.pth", "vgg16_bn": "vgg16_bn-6c64b313.pth",
    "vgg19_bn": "vgg19_bn-c79401a0.pth", "densenet121": "densenet121-a639ec97.pth",
    "densenet161": "densenet161-8d451a50.pth", "densenet169": "densenet169-b2777c0a.pth",
    "densenet201": "densenet201-c1103571.pth", "mobilenet_v2": "mobilenet_v2-b0353104.pth",
    "squeezenet1_0": "squeezenet1_0-b66bff10.pth", "squeezenet1_1": "squeezenet1_1-b8a52dc0.pth",
    "googlenet": "googlenet-1378be20.pth", "inception_v3": "inception_v3_google-0cc3c7bd.pth",
    "shufflenet_v2_x0_5": "shufflenetv2_x0.5-f707e7126e.pth",
    "shufflenet_v2_x1_0": "shufflenetv2_x1-5666bf0f80.pth",
    "mnasnet0_5": "mnasnet0.5_top1_67.823-3ffadce67e.pth",
    "mnasnet1_0": "mnasnet1.0_top1_73.512-f206786ef8.pth",
}


def load_pretrained(model, path: str, strict: bool = True):
    """Load a torchvision state_dict into a mipipe model (identical parameter / buffer names).
    Weights-only loader: nothing in the file is executed."""
    import torch
    sd = torch.load(path, map_location="cpu", weights_only=True)
    if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
        sd = sd["state_dict"]  # a checkpoint written by task.py's save path
    sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
    missing, unexpected = model.load_state_dict(sd, strict=strict)
    return missing, unexpected
