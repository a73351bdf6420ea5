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
    hits = sorted(glob.glob(os.path.join(home, "hub", "checkpoints", f"{arch}-*.pth")))
    return hits[0] if hits else None


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
