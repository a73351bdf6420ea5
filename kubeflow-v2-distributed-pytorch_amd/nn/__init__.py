"""Layers with torch.nn-compatible state (same parameter/buffer names and shapes), executed
by mipipe's fused kernels.

Checkpoints therefore stay interchangeable with torchvision / torch.nn models (the reference
saves ``model.state_dict()``, task.py:282-294).  Differences in *execution*:

* activations are NHWC in the model's compute dtype (bf16 on MI355X);
* conv weights are stored ``channels_last`` so their physical order is ``[Cout,KH,KW,Cin]``,
  the K-contiguous operand layout the implicit-GEMM kernels read;
* each weighted layer reads a compute-dtype *shadow* of its fp32 master weight, refreshed by
  the fused optimizer step (:mod:`mipipe.optim`) instead of a per-layer cast each forward.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn as tnn

from mipipe.ops import functional as MF
from mipipe.ops import kernels as K

__all__ = ["Conv2d", "BatchNorm2d", "Linear", "ReLU", "MaxPool2d", "AdaptiveAvgPool2d",
           "Embedding", "LayerNorm", "Dropout", "ShadowMixin", "conv_bn_act", "XConv2d"]


class ShadowMixin:
    """Provides ``compute_weight(dtype)``: the compute-dtype operand view of ``self.weight``."""

    _shadow: Optional[torch.Tensor] = None

    def operand_view(self, w: torch.Tensor) -> torch.Tensor:
        return w

    def compute_weight(self, dtype: torch.dtype) -> torch.Tensor:
        from mipipe.optim.flat import flat_space_for
        fs = flat_space_for(self.weight)
        if fs is not None and fs.shadow is not None and fs.shadow.dtype == dtype:
            fs.sync_shadow(self.weight)
            sh = self.__dict__.get("_shadow")
            if sh is None or sh.data_ptr() != fs.shadow_view(self.weight).data_ptr():
                sh = self.operand_view(fs.shadow_view(self.weight))
                sh = sh if sh.is_contiguous() else None
                self.__dict__["_shadow"] = sh
            if sh is not None:
                return sh
        w = self.operand_view(self.weight.detach())
        if w.dtype == dtype and w.is_contiguous():
            return w
        return w.to(dtype).contiguous()

    def set_shadow(self, t: Optional[torch.Tensor]) -> None:
        self.__dict__["_shadow"] = t


class Conv2d(ShadowMixin, tnn.Module):
    """``torch.nn.Conv2d``-compatible (groups=1, dilation=1, square kernel/stride/pad)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: int, stride: int = 1,
                 padding: int = 0, bias: bool = False):
        super().__init__()
        k = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = (k, k)
        self.stride = (stride, stride) if isinstance(stride, int) else tuple(stride)
        self.padding = (padding, padding) if isinstance(padding, int) else tuple(padding)
        w = torch.empty(out_channels, in_channels, k, k).to(memory_format=torch.channels_last)
        self.weight = tnn.Parameter(w)
        self.bias = tnn.Parameter(torch.zeros(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self) -> None:
        tnn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            fan_in = self.in_channels * self.kernel_size[0] * self.kernel_size[1]
            bound = 1 / math.sqrt(fan_in)
            tnn.init.uniform_(self.bias, -bound, bound)

    def operand_view(self, w):
        return w.permute(0, 2, 3, 1)  # [Co,KH,KW,Ci]; contiguous when w is channels_last

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        # keep channels_last physical order after .to()/.cuda()
        if not self.weight.is_contiguous(memory_format=torch.channels_last):
            self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)
        return r

    def forward(self, x: torch.Tensor, stats_shift: Optional[torch.Tensor] = None, slabs=None,
                prev=None, res_take=None, res_give=None, in_bn=None):
        """x: NHWC.  Returns y, or (y, psum, psumsq) when ``stats_shift`` is given.  ``in_bn``:
        (scale, bias) of a BatchNorm + ReLU folded into this conv (x holds its input y)."""
        w_c = self.compute_weight(x.dtype)
        y, ps, pss = MF.conv2d(x, self.weight, w_c, self.stride[0], self.padding[0], stats_shift,
                               slabs, prev, res_take, res_give, in_bn)
        if self.bias is not None:
            y = y + self.bias.to(y.dtype)
        return y if stats_shift is None else (y, ps, pss)

    def extra_repr(self) -> str:
        return (f"{self.in_channels}, {self.out_channels}, kernel_size={self.kernel_size}, "
                f"stride={self.stride}, padding={self.padding}, bias={self.bias is not None}")


class XConv2d(ShadowMixin, tnn.Conv2d):
    """``torch.nn.Conv2d`` with any groups / kernel / stride / padding (identical state).

    ``forward`` stays torch's own NCHW convolution — the numerics oracle the model zoo's
    ``reference_forward`` runs.  :meth:`run` executes on NHWC activations through mipipe's
    kernels: the MFMA implicit-GEMM conv when the conv is dense (groups 1, square kernel /
    stride / padding, channel counts % 8), the direct grouped / depthwise kernels otherwise.
    The weight is kept ``channels_last`` so its operand view ``[Co, KH, KW, Ci/groups]`` is
    contiguous (the layout both kernel families read)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)

    def operand_view(self, w):
        return w.permute(0, 2, 3, 1)

    def _apply(self, fn, *args, **kwargs):
        r = super()._apply(fn, *args, **kwargs)
        if not self.weight.is_contiguous(memory_format=torch.channels_last):
            self.weight.data = self.weight.data.contiguous(memory_format=torch.channels_last)
        return r

    def dense(self, cin: int) -> bool:
        """Runs on the MFMA implicit-GEMM kernels for an NHWC input with ``cin`` channels."""
        kh, kw = self.kernel_size
        return (self.groups == 1 and self.dilation == (1, 1) and self.padding_mode == "zeros"
                and not isinstance(self.padding, str) and self.stride[0] == self.stride[1]
                and self.padding[0] < kh and self.padding[1] < kw
                and cin % 8 == 0 and self.out_channels % 8 == 0)

    def mfma_pad(self):
        """Padding argument of the MFMA kernels: an int, or (h, w) for 1xn / nx1 convs."""
        ph, pw = self.padding
        return ph if ph == pw else (ph, pw)

    def kernel_weight(self, dtype: torch.dtype, cin: int) -> torch.Tensor:
        """Operand weight; input channels zero-padded to ``cin`` (padded NHWC stem input)."""
        w = self.compute_weight(dtype)
        if self.groups == 1 and w.shape[-1] < cin:
            w = torch.nn.functional.pad(w, (0, cin - w.shape[-1])).contiguous()
        return w

    def run(self, x: torch.Tensor, act: str = "none") -> torch.Tensor:
        """act(conv(x) + bias) on NHWC ``x``; act in {none, relu, relu6}."""
        if self.dilation != (1, 1) or self.padding_mode != "zeros" or isinstance(self.padding, str):
            raise NotImplementedError("XConv2d.run: dilation / padding modes other than zeros")
        cin = x.shape[-1]
        w_c = self.kernel_weight(x.dtype, cin)
        if self.dense(cin) and act in ("none", "relu"):
            if self.bias is not None or act == "relu":
                return MF.conv2d_bias_act(x, self.weight, w_c, self.bias, self.stride[0],
                                          self.mfma_pad(), act == "relu")
            return MF.conv2d(x, self.weight, w_c, self.stride[0], self.mfma_pad())[0]
        kh, kw = self.kernel_size
        gb = MF.grouped_conv_mfma_blocks(self.groups, w_c.shape[-1],
                                         self.out_channels // self.groups)
        if (gb and act == "none" and self.bias is None and self.stride[0] == self.stride[1]
                and self.padding[0] < kh and self.padding[1] < kw):
            # ResNeXt-style groups (4..64 channels): block-diagonal dense convs on the MFMA
            return MF.block_group_conv2d(x, self.weight, w_c, self.stride[0], self.mfma_pad(),
                                         self.groups, gb)
        return MF.gconv2d(x, self.weight, w_c, self.bias, self.stride, self.padding,
                          self.groups, act)


class BatchNorm2d(tnn.BatchNorm2d):
    """Same state as ``torch.nn.BatchNorm2d``; standalone forward on NHWC input."""

    def forward(self, y: torch.Tensor) -> torch.Tensor:  # NHWC
        training = self.training and self.track_running_stats is not None
        use_batch = self.training or not self.track_running_stats
        if use_batch:
            ps, pss = MF.channel_partials(y, self.running_mean if self.running_mean is not None
                                          else torch.zeros(y.shape[-1], device=y.device))
            st = MF.bn_stats_from_partials(ps, pss, y.numel() // y.shape[-1], self, True)
        else:
            st = MF.bn_stats_from_partials(None, None, y.numel() // y.shape[-1], self, False)
        return MF.batchnorm_act(y, st, self, relu=False)


# Folding BN2 into conv3 saves a read + write of the BN output but costs the conv3 forward /
# weight-grad an in-place LDS transform pass per k-step (+ a barrier and the coefficient table).
# Measured (profiles/r6_bn_fold_negative.txt): per kernel it pays only on ResNet-50 layer 1, and
# end to end it LOSES in every mode — per-fragment transform 12,700 vs 13,150 img/s, LDS-pass
# transform 13,130 vs 13,275 ("1"), size-gated 13,209 vs 13,270 ("auto": tensors of at least
# MIPIPE_BN_FOLD_MIN_ELEMS = 2^25 elements) — so it is off by default ("0").
_BN_FOLD_MODE = os.environ.get("MIPIPE_BN_FOLD", "0")
_BN_FOLD = _BN_FOLD_MODE != "0"
_BN_FOLD_MIN = int(os.environ.get("MIPIPE_BN_FOLD_MIN_ELEMS", str(1 << 25)))


def _foldable_into_1x1(y: torch.Tensor) -> bool:
    """A BN + ReLU output the next dense 1x1 conv can consume folded (bf16 GPU, C <= 1024)."""
    from mipipe.ops import kernels as K
    if not (_BN_FOLD and y.is_cuda and y.dtype == torch.bfloat16 and K.use_native(y)
            and y.shape[-1] <= 1024 and y.shape[-1] % 8 == 0):
        return False
    return _BN_FOLD_MODE == "1" or y.numel() >= _BN_FOLD_MIN


def conv_bn_act(x: torch.Tensor, conv: Conv2d, bn: BatchNorm2d, relu: bool = True,
                residual: Optional[torch.Tensor] = None,
                branch: Optional[tuple] = None, fuse_prev: bool = False,
                res_take: Optional[MF.ResidualSlot] = None,
                res_give: Optional[MF.ResidualSlot] = None,
                fold_next: bool = False) -> torch.Tensor:
    """Fused conv -> BN -> [+residual | +BN(conv(branch_x))] -> ReLU on NHWC activations.

    ``branch`` = (x_b, conv_b, bn_b): the ResNet downsample path, normalised and added in the
    same elementwise pass as the main path.
    ``fuse_prev``: the caller guarantees this conv is the ONLY consumer of ``x`` (an output of
    a previous relu-only conv_bn_act) -> that BN's backward reductions run in this conv's
    dgrad epilogue.  ``res_take`` / ``res_give``: residual-gradient hand-off (the conv that
    also reads the block input adds the identity/downsample gradient in its dgrad epilogue).
    ``fold_next``: the caller guarantees the returned tensor's ONLY consumer is a dense 1x1
    stride-1 conv reached through ``conv_bn_act(fuse_prev=True)`` (ResNet Bottleneck conv3): this
    BN's apply + ReLU is then folded into that conv — its forward and weight-grad read y and
    transform their operand fragments (gemm_core.hpp KCDenseBufBN / MCDenseBufBN), so the
    normalised activation is never written (saves a read and a write of the tensor per step; large
    tensors only by default, see _BN_FOLD_MODE).  The returned tensor is then an alias of y.
    """
    use_batch = bn.training
    prev = getattr(x, "_mipipe_bnact", None) if fuse_prev else None
    in_bn = getattr(x, "_mipipe_lazy_bn", None) if fuse_prev else None
    if in_bn is not None and prev is None:
        raise RuntimeError("a folded BN output reached a conv without its BN token")
    if use_batch:
        ws = MF.bn_workspace(bn, "fwd", x.device)
        y, ps, pss = conv(x, bn.running_mean, None if ws is None else (ws[0], ws[1]), prev=prev,
                          res_take=res_take, in_bn=in_bn)
    else:
        y, ps, pss = conv(x, prev=prev, res_take=res_take, in_bn=in_bn), None, None
    count = y.numel() // y.shape[-1]
    st = MF.bn_stats_from_partials(ps, pss, count, bn, use_batch)
    if branch is not None:
        xb, convb, bnb = branch
        if bnb.training:
            wsb = MF.bn_workspace(bnb, "fwd", xb.device)
            yb, psb, pssb = convb(xb, bnb.running_mean, None if wsb is None else (wsb[0], wsb[1]),
                                  res_give=res_give)
        else:
            yb, psb, pssb = convb(xb, res_give=res_give), None, None
        stb = MF.bn_stats_from_partials(psb, pssb, count, bnb, bnb.training)
        token = None
        if relu and use_batch and bnb.training:
            # the block output's consumer (next block's conv1, which also adds the identity
            # gradient) reduces both BNs' backward in its dgrad epilogue (two-branch fusion)
            token = MF.BNActToken(bn, st, y)
            token.y2, token.st2, token.bn2 = yb, stb, bnb
        z = MF.batchnorm_act(y, st, bn, relu, y2=yb, st2=stb, bn2=bnb, token=token)
        if token is not None:
            token.z = z
            z._mipipe_bnact = token
        return z
    token = None
    if relu and use_batch:
        token = MF.BNActToken(bn, st, y)
    lazy = (fold_next and token is not None and residual is None and torch.is_grad_enabled()
            and _foldable_into_1x1(y))
    z = MF.batchnorm_act(y, st, bn, relu, residual=residual, token=token,
                         res_give=res_give if residual is not None else None, lazy=lazy)
    if token is not None:
        if residual is not None:
            token.z = z  # mask source for the (multi-consumer) block-output fusion
        z._mipipe_bnact = token
    if lazy:
        z._mipipe_lazy_bn = (st.scale, st.bias)
    return z


class ReLU(tnn.ReLU):
    pass


def conv_bn_relu_maxpool(x: torch.Tensor, conv: Conv2d, bn: BatchNorm2d,
                         pool: "MaxPool2d") -> torch.Tensor:
    """maxpool(relu(bn(conv(x)))) — the ResNet stem — with BN-apply, ReLU and the pool in one
    kernel (the normalised activation is never stored) and a gather-based fused backward."""
    if pool.ceil_mode or pool.dilation not in (1, (1, 1)):
        return pool(conv_bn_act(x, conv, bn, relu=True))
    fused = getattr(conv, "fused_bn_relu_maxpool", None)
    if fused is not None:  # packed stem: recompute-fused kernels, conv output never stored
        out = fused(x, bn, *pool.geometry())
        if out is not None:
            return out
    use_batch = bn.training
    if use_batch:
        ws = MF.bn_workspace(bn, "fwd", x.device)
        y, ps, pss = conv(x, bn.running_mean, None if ws is None else (ws[0], ws[1]))
    else:
        y, ps, pss = conv(x), None, None
    st = MF.bn_stats_from_partials(ps, pss, y.numel() // y.shape[-1], bn, use_batch)
    k, s, p = pool.geometry()
    return MF.bn_relu_maxpool(y, st, bn, k, s, p)


class MaxPool2d(tnn.MaxPool2d):
    def geometry(self):
        k = self.kernel_size if isinstance(self.kernel_size, int) else self.kernel_size[0]
        s = self.stride if isinstance(self.stride, int) else self.stride[0]
        p = self.padding if isinstance(self.padding, int) else self.padding[0]
        return k, s, p

    def forward(self, x):  # NHWC
        return MF.max_pool2d(x, *self.geometry())


class AdaptiveAvgPool2d(tnn.AdaptiveAvgPool2d):
    def forward(self, x):  # NHWC -> [N, C]
        return MF.global_avg_pool(x)


class Linear(ShadowMixin, tnn.Linear):
    """``torch.nn.Linear`` state; GEMM on the MFMA kernel with the bias in the epilogue."""

    def forward(self, x: torch.Tensor, act: str = "none", res_take=None,
                bias_slot=None) -> torch.Tensor:
        w_c = self.compute_weight(x.dtype)
        b = None if self.bias is None else self.bias
        return MF.linear(x, self.weight, w_c, b, act, res_take=res_take, bias_slot=bias_slot)


class Embedding(ShadowMixin, tnn.Embedding):
    def forward(self, idx: torch.Tensor, dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        return MF.embedding(idx, self.weight, self.compute_weight(dtype or self.weight.dtype))


class LayerNorm(tnn.LayerNorm):
    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                res_give=None, dropout_p: float = 0.0, dropout_seed=None,
                bias_slot=None) -> torch.Tensor:
        """LN(dropout(x) [+ residual]); the dropout is fused into the LayerNorm kernels
        (``bias_slot``: see :func:`mipipe.ops.functional.layer_norm`)."""
        return MF.layer_norm(x, self.weight, self.bias, self.eps, residual, res_give,
                             dropout_p, dropout_seed, bias_slot)


class Dropout(tnn.Dropout):
    pass
