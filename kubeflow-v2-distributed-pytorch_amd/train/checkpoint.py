"""Model export and training checkpoints.

* ``export_model`` — the reference's export (task.py:282-294): ``torch.save(model.state_dict())``
  of the (DDP-wrapped, hence ``module.``-prefixed) model, to ``<model_dir>/<file>`` with
  ``--local_training`` or to ``AIP_MODEL_DIR/<file>`` otherwise (``AIP_MODEL_DIR/model/<file>``
  with ``--compat-nested-model-dir``, the reference's doubled path).  ``gs://`` destinations go
  to the local object store.  The payload loads into torchvision-layout models after stripping
  the prefix (:func:`strip_module_prefix`).
* ``save_checkpoint`` / ``load_checkpoint`` — the ImageNet-example format the reference's
  resume code expects (task.py:232-238): ``{'epoch','arch','best_acc1','state_dict',
  'optimizer'}``, loaded with ``weights_only=True``.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, Optional

import torch

from mipipe.storage.gcs import uri_to_local_path

__all__ = ["export_model", "save_checkpoint", "load_checkpoint", "load_model_state",
           "strip_module_prefix", "resolve_resume_path", "write_json", "CHECKPOINT_NAME"]

CHECKPOINT_NAME = "checkpoint.pth.tar"


def _atomic_save(obj: Any, path: str) -> None:
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def write_json(path: str, obj: Any) -> None:
    path = uri_to_local_path(path)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(obj, f, indent=2)


def _cpu_state_dict(model) -> Dict[str, torch.Tensor]:
    return {k: v.detach().to("cpu").clone() for k, v in model.state_dict().items()}


def export_model(model, args, epoch: int, accuracy: Optional[float] = None) -> str:
    sd = _cpu_state_dict(model)
    if args.local_training or not os.environ.get("AIP_MODEL_DIR"):
        base = args.model_dir or "."
        path = os.path.join(uri_to_local_path(base), args.model_filename)
    else:
        base = os.environ["AIP_MODEL_DIR"]
        parts = [base, "model", args.model_filename] if args.compat_nested_model_dir else \
            [base, args.model_filename]
        path = uri_to_local_path(os.path.join(*parts))
    _atomic_save(sd, path)
    print(f"saved model (epoch {epoch}, accuracy {accuracy}) to {path}", flush=True)
    return path


def _ckpt_dir(args) -> str:
    base = args.model_dir or os.environ.get("AIP_CHECKPOINT_DIR") or "."
    return uri_to_local_path(base)


def _inner(model):
    return getattr(model, "module", model)


def save_checkpoint(model, optimizer, args, epoch: int, best_acc1: float) -> str:
    state = {"epoch": epoch, "arch": args.arch, "best_acc1": float(best_acc1),
             "state_dict": _cpu_state_dict(model), "optimizer": optimizer.state_dict()}
    step = getattr(_inner(model), "_step", None)
    if isinstance(step, int):
        # the model's dropout-seed step (BERT): a resumed run continues the mask sequence
        # instead of replaying it from step 1
        state["model_step"] = step
    path = os.path.join(_ckpt_dir(args), CHECKPOINT_NAME)
    _atomic_save(state, path)
    return path


def restore_model_step(model, state: Dict[str, Any]) -> None:
    if "model_step" in state and hasattr(_inner(model), "_step"):
        _inner(model)._step = int(state["model_step"])


def resolve_resume_path(resume: str, model_dir: str) -> str:
    if resume == "auto":
        return os.path.join(uri_to_local_path(model_dir or "."), CHECKPOINT_NAME)
    return uri_to_local_path(resume)


def load_checkpoint(path: str, device) -> Dict[str, Any]:
    return torch.load(path, map_location=device, weights_only=True)


def strip_module_prefix(sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    return {(k[len("module."):] if k.startswith("module.") else k): v for k, v in sd.items()}


def load_model_state(model, sd: Dict[str, torch.Tensor], strict: bool = True) -> None:
    """Load a state dict saved with or without the DDP ``module.`` prefix."""
    target_prefixed = any(k.startswith("module.") for k in model.state_dict())
    src_prefixed = any(k.startswith("module.") for k in sd)
    if src_prefixed and not target_prefixed:
        sd = strip_module_prefix(sd)
    elif target_prefixed and not src_prefixed:
        sd = {"module." + k: v for k, v in sd.items()}
    model.load_state_dict(sd, strict=strict)
