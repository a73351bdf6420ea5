"""Fused flat-buffer optimizers.

``SGD`` reproduces ``torch.optim.SGD(params, lr, momentum=0.9, weight_decay=1e-4)`` as used
by the reference (task.py:212-214; update rule [torch] optim/sgd.py:354-380: ``g += wd·p``,
``buf = m·buf + (1-dampening)·g`` (``buf = g`` on the first step), ``p -= lr·buf``), with no
param groups, so weight decay also hits BN affine params and biases exactly like the
reference.  ``AdamW`` is the BERT optimizer.

Both run ONE HIP kernel over the model's flat fp32 parameter buffer
(:class:`~mipipe.optim.flat.FlatParamSpace`) that also rewrites the bf16 compute shadow.
``state_dict()`` uses torch.optim's format (``{'state': {i: {'momentum_buffer': ..}},
'param_groups': [...]}``) so checkpoints are interchangeable with torch.optim.SGD.
"""
from __future__ import annotations

import math
from typing import Any, Dict, Iterable, List, Optional

import torch

from mipipe.ops import kernels as K
from .flat import FlatParamSpace, get_flat_space, flat_space_for

__all__ = ["SGD", "AdamW", "FlatParamSpace", "get_flat_space", "flat_space_for"]


def _default_shadow_dtype(params: List[torch.Tensor]) -> Optional[torch.dtype]:
    return torch.bfloat16 if params and params[0].is_cuda else None


class _FlatOptimizer(torch.optim.Optimizer):
    def __init__(self, params: Iterable, defaults: Dict[str, Any],
                 shadow_dtype: Optional[torch.dtype] = "auto"):
        params = list(params)
        if params and isinstance(params[0], dict):
            if len(params) != 1:
                raise ValueError("mipipe fused optimizers take one param group")
            group_params = list(params[0]["params"])
            defaults = dict(defaults, **{k: v for k, v in params[0].items() if k != "params"})
        else:
            group_params = params
        super().__init__(group_params, defaults)
        if shadow_dtype == "auto":
            shadow_dtype = _default_shadow_dtype(group_params)
        self.space: FlatParamSpace = get_flat_space(group_params, shadow_dtype)

    @property
    def params(self) -> List[torch.Tensor]:
        return self.param_groups[0]["params"]

    def zero_grad(self, set_to_none: bool = True) -> None:  # grads stay flat views
        self.space.zero_grad()

    def _flat_state(self, name: str) -> torch.Tensor:
        st = self.__dict__.setdefault("_flat", {})
        if name not in st:
            st[name] = torch.zeros_like(self.space.flat)
        return st[name]

    def _per_param_state(self, names: List[str]) -> None:
        """Expose flat state as per-parameter views in ``self.state`` (torch format)."""
        from .flat import _view
        for p in self.params:
            d = self.state[p]
            for n in names:
                d[n] = _view(self._flat_state(n), self.space.offset(p), p)

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        super().load_state_dict(state_dict)
        # torch re-creates state tensors; copy them back into the flat buffers
        from .flat import _view
        for p in self.params:
            for n, v in list(self.state[p].items()):
                if torch.is_tensor(v) and v.numel() == p.numel() and n != "step":
                    _view(self._flat_state(n), self.space.offset(p), p).copy_(v.reshape(p.shape))
                    self.state[p][n] = _view(self._flat_state(n), self.space.offset(p), p)
        self._after_load()

    def _after_load(self) -> None:
        pass


class SGD(_FlatOptimizer):
    def __init__(self, params, lr: float = 0.1, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, maximize: bool = False,
                 shadow_dtype="auto"):
        if nesterov and (momentum <= 0 or dampening != 0):
            raise ValueError("Nesterov momentum requires a momentum and zero dampening")
        defaults = dict(lr=lr, momentum=momentum, dampening=dampening,
                        weight_decay=weight_decay, nesterov=nesterov, maximize=maximize,
                        foreach=None, differentiable=False, fused=True)
        super().__init__(params, defaults, shadow_dtype)
        self._steps = 0

    def _after_load(self) -> None:
        if any("momentum_buffer" in self.state[p] for p in self.params):
            self._steps = max(self._steps, 1)

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        if g["maximize"]:
            grad_scale = -grad_scale
        mom = self._flat_state("momentum_buffer") if g["momentum"] != 0 else self.space.flat_grad
        K.sgd_step(self.space.flat, self.space.flat_grad, mom, self.space.shadow, float(g["lr"]),
                   float(g["momentum"]), float(g["dampening"]), float(g["weight_decay"]),
                   bool(g["nesterov"]), self._steps == 0, float(grad_scale))
        self.space.mark_synced()
        self._steps += 1
        if g["momentum"] != 0 and self._steps == 1:
            self._per_param_state(["momentum_buffer"])
        return loss


class AdamW(_FlatOptimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, shadow_dtype="auto"):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                        amsgrad=False, maximize=False, foreach=None, capturable=False,
                        differentiable=False, fused=True)
        super().__init__(params, defaults, shadow_dtype)
        self._step = 0
        # On the GPU the step count also lives on the device (int32 [1]): a device op advances it
        # and the kernel derives the bias corrections 1 - beta^t from it, so a step captured
        # into a hipGraph stays correct on every replay (train/graph.py graph_safe).
        self._t_dev: Optional[torch.Tensor] = None
        self.device_step = self.space.flat.is_cuda

    def _after_load(self) -> None:
        for p in self.params:
            s = self.state[p].get("step")
            if s is not None:
                self._step = int(s.item() if torch.is_tensor(s) else s)
                break
        self._t_dev = None  # re-seeded from the loaded count at the next step

    def sync_step(self) -> int:
        """Host view of the step count (after graph replays the device counter is ahead)."""
        if self._t_dev is not None:
            self._step = int(self._t_dev.item())
            for p in self.params:
                self.state[p]["step"] = torch.tensor(float(self._step))
        return self._step

    def state_dict(self):
        self.sync_step()
        return super().state_dict()

    @torch.no_grad()
    def step(self, closure=None, grad_scale: float = 1.0):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        self._step += 1
        b1, b2 = g["betas"]
        tdev = None
        if self.device_step:
            if self._t_dev is None:
                self._t_dev = torch.full((1,), self._step - 1, dtype=torch.int32,
                                         device=self.space.flat.device)
            self._t_dev.add_(1)
            tdev = self._t_dev
        K.adamw_step(self.space.flat, self.space.flat_grad, self._flat_state("exp_avg"),
                     self._flat_state("exp_avg_sq"), self.space.shadow, float(g["lr"]),
                     float(b1), float(b2), float(g["eps"]), float(g["weight_decay"]),
                     self._step, float(grad_scale), step_dev=tdev)
        self.space.mark_synced()
        if self._step == 1:
            self._per_param_state(["exp_avg", "exp_avg_sq"])
        for p in self.params:
            self.state[p]["step"] = torch.tensor(float(self._step))
        return loss
