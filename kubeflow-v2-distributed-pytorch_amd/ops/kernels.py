"""Kernel entry points: HIP (``mipipe._C``) for GPU tensors, ATen reference for CPU tensors.

GPU tensors always go to the hand-written gfx950 kernels.  If the extension is missing on
a GPU box the call raises (no silent fallback to stock torch kernels), unless the caller
opted in with ``MIPIPE_ALLOW_REF_ON_GPU=1`` (debugging / numerics bisection only).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from . import _ref
from ._native import native, native_available

__all__ = ["conv_fwd", "conv_dgrad", "conv_wgrad", "bn_finalize", "bn_act_fwd",
           "bn_act_bwd_reduce", "bn_act_bwd_apply", "maxpool_fwd", "maxpool_bwd",
           "avgpool_fwd", "avgpool_bwd", "gemm", "cross_entropy_fwd_bwd", "sgd_step",
           "adamw_step", "layernorm_fwd", "layernorm_bwd", "attention_fwd", "attention_bwd",
           "embedding_bwd", "gelu_fwd", "gelu_bwd", "nchw_to_nhwc", "use_native"]

_ALLOW_REF_ON_GPU = os.environ.get("MIPIPE_ALLOW_REF_ON_GPU", "0") == "1"


def use_native(t: torch.Tensor) -> bool:
    if not t.is_cuda:
        return False
    if native_available():
        return True
    if _ALLOW_REF_ON_GPU:
        return False
    raise RuntimeError(
        "mipipe._C (gfx950 HIP kernels) is not built/loadable but a GPU tensor reached a "
        "mipipe op.  Run `python -c 'import __graft_entry__ as g; g.build()'` (or "
        "`python setup.py build_ext --inplace`).  Set MIPIPE_ALLOW_REF_ON_GPU=1 only to debug.")


def conv_fwd(x, w, stride, pad, stats_shift=None):
    if use_native(x):
        return native().conv_fwd(x, w, stride, pad, stats_shift)
    return _ref.conv_fwd(x, w, stride, pad, stats_shift)


def conv_dgrad(dy, w, x_shape, stride, pad):
    if use_native(dy):
        return native().conv_dgrad(dy, w, list(x_shape), stride, pad)
    return _ref.conv_dgrad(dy, w, x_shape, stride, pad)


def conv_wgrad(dy, x, kh, kw, stride, pad):
    if use_native(dy):
        return native().conv_wgrad(dy, x, kh, kw, stride, pad)
    return _ref.conv_wgrad(dy, x, kh, kw, stride, pad)


def bn_finalize(psum, psumsq, count, shift, gamma, beta, running_mean, running_var,
                momentum, eps):
    if use_native(psum):
        return native().bn_finalize(psum, psumsq, count, shift, gamma, beta, running_mean,
                                    running_var, momentum, eps)
    return _ref.bn_finalize(psum, psumsq, count, shift, gamma, beta, running_mean,
                            running_var, momentum, eps)


def bn_act_fwd(y, scale, bias, relu, residual=None, res_scale=None, res_bias=None):
    if use_native(y):
        return native().bn_act_fwd(y, scale, bias, relu, residual, res_scale, res_bias)
    return _ref.bn_act_fwd(y, scale, bias, relu, residual, res_scale, res_bias)


def bn_act_bwd_reduce(dz, z, y, mean, invstd, relu, y2=None, mean2=None, invstd2=None):
    """Returns (Σg, Σg·x̂) for y and, when ``y2`` is given (downsample branch sharing the same
    add/ReLU), (Σg·x̂2) for y2 as a third output."""
    if use_native(dz):
        return native().bn_act_bwd_reduce(dz, z, y, mean, invstd, relu, y2, mean2, invstd2)
    sg, sgx = _ref.bn_act_bwd_reduce(dz, z, y, mean, invstd, relu)
    if y2 is None:
        return sg, sgx, None
    _, sgx2 = _ref.bn_act_bwd_reduce(dz, z, y2, mean2, invstd2, relu)
    return sg, sgx, sgx2


def bn_act_bwd_apply(dz, z, y, mean, invstd, gamma, sum_g, sum_gx, count, relu,
                     want_dres=False, y2=None, mean2=None, invstd2=None, gamma2=None,
                     sum_gx2=None):
    """Returns (dy, dres_or_dy2): dres = g when ``want_dres``; dy2 = BN-bwd of y2 when ``y2``."""
    if use_native(dz):
        return native().bn_act_bwd_apply(dz, z, y, mean, invstd, gamma, sum_g, sum_gx, count,
                                         relu, want_dres, y2, mean2, invstd2, gamma2, sum_gx2)
    dy, dres = _ref.bn_act_bwd_apply(dz, z, y, mean, invstd, gamma, sum_g, sum_gx, count, relu,
                                     want_dres)
    if y2 is not None:
        dy2, _ = _ref.bn_act_bwd_apply(dz, z, y2, mean2, invstd2, gamma2, sum_g, sum_gx2,
                                       count, relu)
        return dy, dy2
    return dy, dres


def maxpool_fwd(x, k, stride, pad):
    if use_native(x):
        return native().maxpool_fwd(x, k, stride, pad)
    return _ref.maxpool_fwd(x, k, stride, pad)


def maxpool_bwd(dy, idx, x_shape, k, stride, pad):
    if use_native(dy):
        return native().maxpool_bwd_impl(dy, idx, list(x_shape), k, stride, pad)
    return _ref.maxpool_bwd(dy, idx, x_shape)


def avgpool_fwd(x):
    if use_native(x):
        return native().avgpool_fwd(x)
    return _ref.avgpool_fwd(x)


def avgpool_bwd(dy, x_shape):
    if use_native(dy):
        return native().avgpool_bwd(dy, list(x_shape))
    return _ref.avgpool_bwd(dy, x_shape)


def gemm(a, b, trans_a=False, trans_b=False, bias=None, act="none", out_dtype=None, c=None,
         beta=0.0):
    if use_native(a):
        return native().gemm(a, b, trans_a, trans_b, bias, act,
                             out_dtype if out_dtype is not None else a.dtype, c, beta)
    return _ref.gemm(a, b, trans_a, trans_b, bias, act, out_dtype, c, beta)


def cross_entropy_fwd_bwd(logits, labels, label_smoothing=0.0, ignore_index=-100):
    if use_native(logits):
        return native().cross_entropy_fwd_bwd(logits, labels, label_smoothing, ignore_index)
    return _ref.cross_entropy_fwd_bwd(logits, labels, label_smoothing, ignore_index)


def sgd_step(param, grad, mom, shadow, lr, momentum, dampening, weight_decay, nesterov,
             first_step, grad_scale=1.0):
    if use_native(param):
        return native().sgd_step(param, grad, mom, shadow, lr, momentum, dampening,
                                 weight_decay, nesterov, first_step, grad_scale)
    return _ref.sgd_step(param, grad, mom, shadow, lr, momentum, dampening, weight_decay,
                         nesterov, first_step, grad_scale)


def adamw_step(param, grad, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2, eps, weight_decay,
               step, grad_scale=1.0):
    if use_native(param):
        return native().adamw_step(param, grad, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2,
                                   eps, weight_decay, step, grad_scale)
    return _ref.adamw_step(param, grad, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2, eps,
                           weight_decay, step, grad_scale)


def layernorm_fwd(x, gamma, beta, eps, residual=None):
    if use_native(x):
        return native().layernorm_fwd(x, gamma, beta, eps, residual)
    return _ref.layernorm_fwd(x, gamma, beta, eps, residual)


def layernorm_bwd(dy, x, mean, rstd, gamma):
    if use_native(dy):
        return native().layernorm_bwd(dy, x, mean, rstd, gamma)
    return _ref.layernorm_bwd(dy, x, mean, rstd, gamma)


def attention_fwd(q, k, v, mask_bias, scale):
    if use_native(q):
        return native().attention_fwd(q, k, v, mask_bias, scale)
    return _ref.attention_fwd(q, k, v, mask_bias, scale)


def attention_bwd(do, q, k, v, o, lse, mask_bias, scale):
    if use_native(do):
        return native().attention_bwd(do, q, k, v, o, lse, mask_bias, scale)
    return _ref.attention_bwd(do, q, k, v, o, lse, mask_bias, scale)


def embedding_bwd(dy, idx, num_rows):
    if use_native(dy):
        return native().embedding_bwd(dy, idx, num_rows)
    return _ref.embedding_bwd(dy, idx, num_rows)


def gelu_fwd(x):
    if use_native(x):
        return native().gelu_fwd(x)
    return _ref.gelu_fwd(x)


def gelu_bwd(dy, x):
    if use_native(dy):
        return native().gelu_bwd(dy, x)
    return _ref.gelu_bwd(dy, x)


def nchw_to_nhwc(x, dtype, pad_channels_to: int = 0):
    """[N,C,H,W] (any float) -> [N,H,W,C'] ``dtype``, C' = C zero-padded up to a multiple of
    ``pad_channels_to`` (the stem conv wants Cin % 8 == 0 for 16-byte MFMA operand loads)."""
    if use_native(x):
        return native().nchw_to_nhwc(x, dtype, pad_channels_to)
    y = x.permute(0, 2, 3, 1)
    C = y.shape[-1]
    if pad_channels_to and C % pad_channels_to:
        y = torch.nn.functional.pad(y, (0, pad_channels_to - C % pad_channels_to))
    return y.contiguous().to(dtype)
