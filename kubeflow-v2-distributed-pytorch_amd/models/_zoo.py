"""Shared NHWC executor for the torchvision-structured model zoo (task.py:50-52, 166-171).

The zoo models (MobileNetV2, MNASNet, ShuffleNetV2, SqueezeNet, DenseNet, GoogLeNet,
Inception-v3) keep torchvision's module tree, so ``state_dict`` keys and shapes are
torchvision's and every block's ``forward`` is plain torch on NCHW — the numerics oracle exposed
as ``model.reference_forward``.  Training and inference (``model(x)``) run through
:func:`run_seq` instead: NHWC activations in the compute dtype, every convolution on mipipe's
kernels (MFMA implicit GEMM when dense, the direct grouped / depthwise kernels otherwise), BN
batch statistics accumulated in the producing MFMA conv's epilogue where possible, BN +
ReLU/ReLU6 in one pass and residual adds folded into the BN apply.
"""
from __future__ import annotations

from typing import Optional, Sequence, Tuple

import torch
import torch.nn as tnn
import torch.nn.functional as F

from mipipe import nn as mnn
from mipipe.ops import functional as MF
from mipipe.ops import kernels as K

__all__ = ["ZooModel", "Exec", "run_seq", "run_module", "conv_bn", "act_of", "global_pool",
           "adaptive_avg_pool", "ref_linear"]


class Exec:
    """Per-forward execution context: hash-keyed dropout needs a fresh seed per layer and step."""

    __slots__ = ("base", "n")

    def __init__(self, base: int):
        self.base, self.n = base, 0

    def seed(self) -> int:
        self.n += 1
        return (self.base + self.n * 7919) & 0xFFFFFFFF


def act_of(m) -> str:
    if isinstance(m, tnn.ReLU6):
        return "relu6"
    if isinstance(m, tnn.ReLU):
        return "relu"
    return "none"


def conv_bn(x: torch.Tensor, conv: mnn.XConv2d, bn: tnn.BatchNorm2d, act: str = "relu",
            residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(BN(conv(x)) [+ residual]).  A dense conv accumulates the BN batch statistics in its
    MFMA epilogue and BN (+residual) (+ReLU) is one elementwise pass; other convs run the
    direct kernel, then the any-C BN pass."""
    cin = x.shape[-1]
    if conv.dense(cin) and conv.bias is None and act in ("none", "relu"):
        w_c = conv.kernel_weight(x.dtype, cin)
        s, p = conv.stride[0], conv.mfma_pad()
        if bn.training:
            ws = MF.bn_workspace(bn, "fwd", x.device)
            y, ps, pss = MF.conv2d(x, conv.weight, w_c, s, p, bn.running_mean,
                                   None if ws is None else (ws[0], ws[1]))
        else:
            y, ps, pss = MF.conv2d(x, conv.weight, w_c, s, p)
        st = MF.bn_stats_from_partials(ps, pss, y.numel() // y.shape[-1], bn, bn.training)
        return MF.batchnorm_act(y, st, bn, act == "relu", residual=residual)
    y = conv.run(x, "none")
    if residual is None:
        return MF.bn_act(y, bn, act)
    z = MF.bn_act(y, bn, "none") + residual
    return torch.relu(z) if act == "relu" else z


def _pool_args(m) -> Tuple[int, int, int]:
    k = m.kernel_size if isinstance(m.kernel_size, int) else m.kernel_size[0]
    s = m.stride if isinstance(m.stride, int) else (m.stride[0] if m.stride else k)
    p = m.padding if isinstance(m.padding, int) else m.padding[0]
    return k, s, p


def global_pool(x: torch.Tensor) -> torch.Tensor:
    """NHWC [N, H, W, C] -> [N, C] mean (AdaptiveAvgPool2d(1) + flatten)."""
    if x.shape[-1] % 8 == 0:
        return MF.global_avg_pool(x)
    return x.mean(dim=(1, 2))


def adaptive_avg_pool(x: torch.Tensor, size) -> torch.Tensor:
    size = (size, size) if isinstance(size, int) else tuple(size)
    N, H, W, C = x.shape
    if size == (1, 1):
        return global_pool(x).reshape(N, 1, 1, C)
    if (H, W) == size:
        return x
    xc = x.permute(0, 3, 1, 2)  # uneven windows (e.g. GoogLeNet aux 14x14 -> 4x4): torch op
    y = F.adaptive_avg_pool2d(xc.float() if xc.dtype == torch.bfloat16 else xc, size)
    return y.to(x.dtype).permute(0, 2, 3, 1).contiguous()


def ref_linear(m: tnn.Linear, x: torch.Tensor) -> torch.Tensor:
    """Plain-torch Linear (the reference path never touches mipipe's GEMM kernel)."""
    return F.linear(x, m.weight, m.bias)


def run_module(m: tnn.Module, x: torch.Tensor, ex: Exec) -> torch.Tensor:
    if isinstance(m, mnn.XConv2d):
        return m.run(x)
    if isinstance(m, tnn.BatchNorm2d):
        return MF.bn_act(x, m, "none")
    if isinstance(m, mnn.Linear):
        return m(x)
    run = getattr(m, "run", None)
    if run is not None:
        return run(x, ex)
    if isinstance(m, tnn.Sequential):
        return run_seq(m, x, ex)
    if isinstance(m, tnn.MaxPool2d):
        k, s, p = _pool_args(m)
        return MF.max_pool2d(x, k, s, p, m.ceil_mode)
    if isinstance(m, tnn.AvgPool2d):
        if m.ceil_mode or not m.count_include_pad or m.divisor_override:
            raise NotImplementedError("AvgPool2d: only torch's default modes are supported")
        k, s, p = _pool_args(m)
        return MF.avg_pool2d(x, k, s, p)
    if isinstance(m, tnn.AdaptiveAvgPool2d):
        return adaptive_avg_pool(x, m.output_size)
    if isinstance(m, tnn.ReLU6):
        return x.clamp(0.0, 6.0)
    if isinstance(m, tnn.ReLU):
        return torch.relu(x)
    if isinstance(m, tnn.Dropout):
        return MF.dropout(x, m.p, ex.seed(), m.training)
    if isinstance(m, tnn.Identity):
        return x
    raise TypeError(f"no mipipe execution rule for {type(m).__name__}")


def run_seq(seq: Sequence[tnn.Module], x: torch.Tensor, ex: Exec) -> torch.Tensor:
    """Execute a torchvision Sequential on NHWC activations, fusing Conv[+BN][+ReLU/ReLU6],
    BN[+act] and Linear[+ReLU] groups."""
    mods = list(seq)
    i = 0
    while i < len(mods):
        m = mods[i]
        n1 = mods[i + 1] if i + 1 < len(mods) else None
        n2 = mods[i + 2] if i + 2 < len(mods) else None
        if isinstance(m, mnn.XConv2d) and isinstance(n1, tnn.BatchNorm2d):
            act = act_of(n2)
            x = conv_bn(x, m, n1, act)
            i += 3 if act != "none" else 2
        elif isinstance(m, mnn.XConv2d):
            act = act_of(n1)
            x = m.run(x, act)
            i += 2 if act != "none" else 1
        elif isinstance(m, tnn.BatchNorm2d):
            act = act_of(n1)
            x = MF.bn_act(x, m, act)
            i += 2 if act != "none" else 1
        elif isinstance(m, mnn.Linear):
            relu = isinstance(n1, tnn.ReLU) and not isinstance(n1, tnn.ReLU6)
            x = m(x, act="relu" if relu else "none")
            i += 2 if relu else 1
        else:
            x = run_module(m, x, ex)
            i += 1
    return x


class ZooModel(tnn.Module):
    """Base of the zoo models: compute-dtype choice, NCHW -> NHWC entry, dropout seeds.

    ``forward(x)`` runs mipipe's kernels; ``reference_forward(x)`` runs the identical module
    tree with plain torch ops on NCHW (numerics oracle, same parameters and buffers)."""

    compute_dtype: Optional[torch.dtype] = None
    _step = 0

    def activation_dtype(self, x: torch.Tensor) -> torch.dtype:
        if self.compute_dtype is not None:
            return self.compute_dtype
        return torch.bfloat16 if x.is_cuda else torch.float32

    def begin(self, x: torch.Tensor) -> Tuple[torch.Tensor, Exec]:
        if self.training:
            self._step += 1
        return K.nchw_to_nhwc(x, self.activation_dtype(x), 8), Exec(self._step * 104729)

    def forward(self, x: torch.Tensor):
        return self.run_model(*self.begin(x))

    def run_model(self, x: torch.Tensor, ex: Exec):  # pragma: no cover - abstract
        raise NotImplementedError

    def reference_forward(self, x: torch.Tensor):  # pragma: no cover - abstract
        raise NotImplementedError
