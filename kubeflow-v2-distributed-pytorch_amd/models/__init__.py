"""Model zoo + registry with torchvision-style ``--arch`` semantics (task.py:50-52, 63-67).

``model_names()`` lists the lower-case constructor names, like the reference's scan of
``torchvision.models.__dict__``; ``create_model(arch, **kw)`` builds one.
"""
from __future__ import annotations

from typing import Callable, Dict, List

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
