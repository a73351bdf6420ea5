"""Kernel entry points: HIP (``mipipe._C``) for GPU tensors, ATen reference for CPU tensors.

GPU tensors always go to the hand-written gfx950 kernels.  If the extension is missing on
a GPU box the call raises (no silent fallback to stock torch kernels), unless the caller
opted in with ``MIPIPE_ALLOW_REF_ON_GPU=1`` (debugging / numerics bisection only).
"""
from __future__ import annotations

import os
from typing import NamedTuple, Optional

import torch

from . import _ref
from ._ref import _f
from ._native import native, native_available

__all__ = ["conv_fwd", "conv_dgrad", "conv_wgrad", "bn_finalize", "bn_act_fwd",
           "bn_act_bwd_reduce", "bn_act_bwd_apply", "maxpool_fwd", "maxpool_bwd",
           "avgpool_fwd", "avgpool_bwd", "pool_bn_fwd", "pool_bn_bwd", "pool_bn_supported", "stem_fused_supported", "stem_fwd_stats",
           "stem_fwd_pool", "stem_bwd", "gemm", "cross_entropy_fwd_bwd", "top1_correct", "sgd_step",
           "adamw_step", "layernorm_fwd", "layernorm_bwd", "attention_fwd", "attention_bwd", "dropout_fwd", "colsum", "bn_bwd_collect", "stem_pack",
           "embedding_bwd", "gelu_fwd", "gelu_bwd", "nchw_to_nhwc", "use_native",
           "gconv_fwd", "gconv_dgrad", "gconv_wgrad", "chan_stats", "affine_act",
           "bn_generic_bwd_reduce", "bn_generic_bwd_apply", "avgpool2d_fwd", "avgpool2d_bwd"]

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


def _pads(pad):
    """(vertical, horizontal) padding for the kernels; -1 = same as vertical."""
    return (pad, -1) if isinstance(pad, int) else (int(pad[0]), int(pad[1]))


def conv_fwd(x, w, stride, pad, stats_shift=None, slabs=None, bias=None, relu=False,
             wflip=None, in_bn=None):
    """``slabs``: persistent zeroed (sum, sumsq) replica slabs the GPU epilogue accumulates BN
    statistics into (re-zeroed by :func:`bn_finalize`).  ``bias`` / ``relu``: epilogue bias and
    ReLU for convolutions without BatchNorm (exclusive with the statistics epilogue).
    ``wflip`` (native, :func:`dgrad_preflip_ok` shapes): extra blocks of the same launch write
    the tap-flipped weight the data-grad reads — pass it to :func:`conv_dgrad` as ``wflip``.
    ``in_bn = (scale, bias)``: folded input BatchNorm (bf16 dense 1x1): ``x`` holds y and the conv
    consumes relu(y*scale + bias), the normalised tensor is never written."""
    sh, sw = (stride, 0) if isinstance(stride, int) else (stride[0], stride[1])
    ph, pw = _pads(pad)
    if use_native(x):
        s1, s2 = slabs if slabs is not None else (None, None)
        isc, ibi = in_bn if in_bn is not None else (None, None)
        return native().conv_fwd(x, w, sh, ph, stats_shift, s1, s2, bias, relu, sw, pw,
                                 wflip=wflip, in_scale=isc, in_bias=ibi)
    if in_bn is not None:
        x = _ref.bn_relu_fold(x, *in_bn)
    y, a, b = _ref.conv_fwd(x, w, stride if isinstance(stride, int) else tuple(stride),
                            pad if isinstance(pad, int) else tuple(pad), stats_shift)
    if bias is not None or relu:
        yf = _f(y) if bias is None else _f(y) + _f(bias)
        y = (torch.relu(yf) if relu else yf).to(x.dtype)
    return y, a, b


def dgrad_preflip_ok(x_shape, w_shape, stride, pad) -> bool:
    """The conv forward can write this conv's flipped data-grad weight (stride 1, k > 1)."""
    if not (isinstance(stride, int) and isinstance(pad, int)) or not native_available():
        return False
    return bool(native().dgrad_preflip_ok(list(x_shape), list(w_shape), stride, pad))


def conv_dgrad(dy, w, x_shape, stride, pad, addend=None, bnr=None, bnr2=None, wflip=None):
    """dx of an NHWC conv.  ``addend``: tensor added to dx in the epilogue (residual gradient).
    ``bnr = (y, mean, invstd, scale, bias, rep[, z])``: the conv input was relu(bn(y)[+res]);
    dx becomes g = dx·[z > 0] (z recomputed from y unless given — as the stored tensor, or as
    its uint8 bit mask from ``bn_act_fwd(mask=)``) and Σg, Σg·x̂ accumulate into ``rep`` rows
    0/1 (native only).  ``bnr2 = (y2, mean2, invstd2)``: the input was relu(bn(y) + bn2(y2))
    (ResNet downsample block output): Σg·x̂₂ into ``rep`` array 2 (bf16 1x1 convs)."""
    if use_native(dy):
        ph, pw = _pads(pad)
        if bnr is None:
            return native().conv_dgrad(dy, w, list(x_shape), stride, ph, addend, pad_w=pw,
                                       wflip_pre=wflip)
        y, mean, invstd, scale, bias, rep = bnr[:6]
        z = bnr[6] if len(bnr) > 6 else None
        mask = None
        if z is not None and z.dtype == torch.uint8:
            z, mask = None, z
        y2, mean2, invstd2 = bnr2 if bnr2 is not None else (None, None, None)
        return native().conv_dgrad(dy, w, list(x_shape), stride, ph, addend, y, mean, invstd,
                                   scale, bias, rep, z, pw, bn_mask=mask, bn_y2=y2,
                                   bn_mean2=mean2, bn_invstd2=invstd2, wflip_pre=wflip)
    if bnr is not None:
        raise RuntimeError("BN-reduce dgrad fusion is a native-kernel path")
    dx = _ref.conv_dgrad(dy, w, x_shape, stride, pad if isinstance(pad, int) else tuple(pad))
    return dx if addend is None else (dx + addend).to(dx.dtype)


def bn_bwd_collect(rep, C, acc=None):
    """(Σg, Σg·x̂) from a bwd replica slab filled by a fused dgrad; re-zeroes the slab."""
    a = acc if acc is not None else (None, None)
    return native().bn_bwd_collect(rep, C, *a)


def conv_wgrad(dy, x, kh, kw, stride, pad, out=None, collect=None, in_bn=None):
    """``out``: accumulate into this fp32 [Co,KH,KW,Ci] buffer (the parameter's flat gradient).
    ``stride``: int or (vertical, horizontal).  ``collect = (rep, out2, dgamma, dbeta[, True,
    dgamma2, dbeta2])`` (native): one block of the launch also does :func:`bn_bwd_collect` of
    ``rep`` into ``out2`` [2, C] (Σg, Σg·x̂; dgamma / dbeta accumulators or None) — the slab a
    fused dgrad just filled; the 7-tuple form also collects Σg·x̂₂ (out2 [3, C]).
    ``in_bn``: folded input BatchNorm (see :func:`conv_fwd`)."""
    sh, sw = (stride, 0) if isinstance(stride, int) else (stride[0], stride[1])
    if use_native(dy):
        ph, pw = _pads(pad)
        c = tuple(collect) if collect is not None else (None, None, None, None)
        if len(c) == 4:
            c = c + (False, None, None)
        isc, ibi = in_bn if in_bn is not None else (None, None)
        return native().conv_wgrad(dy, x, kh, kw, sh, ph, out, sw, pw, -1, *c, isc, ibi)
    if collect is not None:
        raise RuntimeError("collect-in-wgrad is a native-kernel path")
    if in_bn is not None:
        x = _ref.bn_relu_fold(x, *in_bn)
    dw = _ref.conv_wgrad(dy, x, kh, kw, stride if isinstance(stride, int) else tuple(stride),
                         pad if isinstance(pad, int) else tuple(pad))
    if out is not None:
        out.add_(dw)
        return out
    return dw


def bn_finalize(psum, psumsq, count, shift, gamma, beta, running_mean, running_var,
                momentum, eps, num_batches_tracked=None):
    """``num_batches_tracked`` (int64 scalar) is incremented by the same kernel."""
    if use_native(psum):
        nbt = num_batches_tracked
        if nbt is not None and (nbt.dtype != torch.int64 or not nbt.is_cuda):
            nbt.add_(1)
            nbt = None
        return native().bn_finalize(psum, psumsq, count, shift, gamma, beta, running_mean,
                                    running_var, momentum, eps, True, nbt)
    if num_batches_tracked is not None:
        num_batches_tracked.add_(1)
    return _ref.bn_finalize(psum, psumsq, count, shift, gamma, beta, running_mean,
                            running_var, momentum, eps)


def bn_act_fwd(y, scale, bias, relu, residual=None, res_scale=None, res_bias=None, mask=None):
    """z = relu?(y*scale + bias [+ residual | + residual*res_scale + res_bias]).  ``mask``
    (native, uint8 [rows, C/8]): also receives z > 0 as bits (bit q of byte c = channel 8c+q),
    the ReLU mask the backward reads instead of z."""
    if use_native(y):
        return native().bn_act_fwd(y, scale, bias, relu, residual, res_scale, res_bias, mask)
    return _ref.bn_act_fwd(y, scale, bias, relu, residual, res_scale, res_bias)


def bn_act_bwd_reduce(dz, z, y, mean, invstd, relu, y2=None, mean2=None, invstd2=None,
                      rep=None, acc=None):
    """Returns (Σg, Σg·x̂) for y and, when ``y2`` is given (downsample branch sharing the same
    add/ReLU), (Σg·x̂2) for y2 as a third output.  ``rep``: persistent zeroed replica slab."""
    if use_native(dz):
        a = acc if acc is not None else (None, None, None, None)
        return native().bn_act_bwd_reduce(dz, z, y, mean, invstd, relu, y2, mean2, invstd2, rep,
                                          *a)
    sg, sgx = _ref.bn_act_bwd_reduce(dz, z, y, mean, invstd, relu)
    sgx2 = None
    if y2 is not None:
        _, sgx2 = _ref.bn_act_bwd_reduce(dz, z, y2, mean2, invstd2, relu)
    if acc is not None:  # same contract as the native kernel: accumulate dγ/dβ in place
        dg, db, dg2, db2 = acc
        dg.add_(sgx.to(dg.dtype))
        db.add_(sg.to(db.dtype))
        if dg2 is not None:
            dg2.add_(sgx2.to(dg2.dtype))
            db2.add_(sg.to(db2.dtype))
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


def maxpool_fwd(x, k, stride, pad, ceil_mode=False):
    if use_native(x):
        return native().maxpool_fwd(x, k, stride, pad, bool(ceil_mode))
    return _ref.maxpool_fwd(x, k, stride, pad, ceil_mode)


def maxpool_bwd(dy, idx, x_shape, k, stride, pad):
    if use_native(dy):
        return native().maxpool_bwd_impl(dy, idx, list(x_shape), k, stride, pad)
    return _ref.maxpool_bwd(dy, idx, x_shape)


def pool_bn_fwd(y, scale, bias, k, stride, pad):
    """(maxpool(relu(y*scale + bias)), window argmax) without storing the normalised
    activation (native; NHWC, C % 8 == 0 and 256 % (C/8) == 0)."""
    return native().pool_bn_fwd(y, scale, bias, k, stride, pad)


def pool_bn_bwd(dp, idx, pout, y, mean, invstd, gamma, rep, count, k, stride, pad, acc=None):
    """Backward of :func:`pool_bn_fwd` + the BN statistics: (dy, Σg, Σg·x̂); ``acc`` = (dγ, dβ)
    accumulators (the flat gradient buffer) or None.  ``rep``: zeroed bwd replica slab."""
    a = acc if acc is not None else (None, None)
    return native().pool_bn_bwd(dp, idx, pout, y, mean, invstd, gamma, rep, count, k, stride, pad,
                                *a)


def stem_fused_supported(xp, w) -> bool:
    """The recompute-fused stem kernels (stem.hip) take this packed input / weight."""
    return use_native(xp) and bool(native().stem_fused_supported(xp, w))


def stem_wgrad_unpack(dwp, g) -> None:
    """g[co][c][kh][kw] += dwp[co][kh][kw // 2][(kw % 2) * 4 + c] (native; g fp32, any strides)."""
    native().stem_wgrad_unpack(dwp, g)


def stem_fwd_stats(xp, w, shift, slab_sum, slab_sq):
    """Shifted Σ, Σ² of the packed stem conv's bf16 output into zeroed replica slabs [R, 64]
    (native; the conv output is recomputed, not stored)."""
    return native().stem_fwd_stats(xp, w, shift, slab_sum, slab_sq)


def stem_fwd_pool(xp, w, scale, bias, want_y=True):
    """(maxpool_3x3/2/1(relu(conv(xp)*scale + bias)), window tap, conv output y or None)
    (native); the tap is 0xFF where the output is not > 0."""
    return native().stem_fwd_pool(xp, w, scale.contiguous(), bias.contiguous(), bool(want_y))


def stem_bwd(xp, y, dp, idx, pout, mean, invstd, gamma, beta, rep, count, acc=None):
    """Backward of the fused stem: (packed dW [64,7,4,8] fp32, Σg, Σg·x̂) — the BN reduction over
    the pooled (dp, output) pair (x̂ = (z-β)/γ where z > 0), then the BN-apply folded into the
    weight-grad; ``acc`` = (dγ, dβ) accumulators or None; ``rep``: zeroed bwd replica slab."""
    a = acc if acc is not None else (None, None)
    return native().stem_bwd(xp, y, dp, idx, pout, mean, invstd, gamma.float().contiguous(),
                             beta.float().contiguous(), rep, int(count), *a)


def pool_bn_supported(y) -> bool:
    C = y.shape[-1]
    return use_native(y) and C % 8 == 0 and 256 % (C // 8) == 0


def avgpool_fwd(x):
    if use_native(x):
        return native().avgpool_fwd(x)
    return _ref.avgpool_fwd(x)


def avgpool_bwd(dy, x_shape):
    if use_native(dy):
        return native().avgpool_bwd(dy, list(x_shape))
    return _ref.avgpool_bwd(dy, x_shape)


def _pad2(t, r, c):
    """Zero-pad a 2-D tensor to [r, c] (no copy when already that shape)."""
    if t.shape[0] == r and t.shape[1] == c:
        return t
    out = t.new_zeros(r, c)
    out[: t.shape[0], : t.shape[1]] = t
    return out


# MIPIPE_GEMM_GELU=1: the GELU in the GEMM epilogue.  Measured neutral on BERT-base (7.296 vs
# 7.277 ms/step, same box, alternating: profiles/r4_gemm_gelu_ab.txt) — the epilogue's erf
# VALU costs what the separate HBM-bound pass did — so off by default.
_GEMM_GELU = os.environ.get("MIPIPE_GEMM_GELU", "0") == "1"


def gemm_gelu_ok(x, w) -> bool:
    """gemm_gelu runs as one native GEMM for x [M, K] @ w [N, K]^T (bf16, multiples of 8)."""
    return (_GEMM_GELU and use_native(x) and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16
            and x.dim() == 2 and w.dim() == 2 and x.shape[1] % 8 == 0 and w.shape[0] % 8 == 0
            and x.is_contiguous() and w.is_contiguous())


def gemm_gelu(x, w, bias=None, prefetch=None):
    """(gelu(x @ w^T + bias), x @ w^T + bias): the GELU Linear forward with the activation in
    the GEMM epilogue (the pre-activation is the backward's saved tensor).  ``prefetch``: as
    :func:`gemm` (the two-launch form only)."""
    if gemm_gelu_ok(x, w):
        return native().gemm_gelu(x, w, bias)
    h = gemm(x, w, False, True, bias, "none", x.dtype, prefetch=prefetch)
    return gelu_fwd(h), h


def gemm(a, b, trans_a=False, trans_b=False, bias=None, act="none", out_dtype=None, c=None,
         beta=0.0, addend=None, prefetch=None):
    """act(op(a) @ op(b) + bias) [+ beta * c] [+ addend]; ``addend`` (same shape / dtype as the
    output; a @ b form, no bias / act) is added in the GEMM epilogue.  ``prefetch``: up to two
    tensors (another GEMM's cold operands) this GEMM's blocks warm into the memory-side cache
    (mipipe/ops/prefetch.py); a hint only, ignored off the native path."""
    if addend is not None:
        M = a.shape[1] if trans_a else a.shape[0]
        N = b.shape[0] if trans_b else b.shape[1]
        Kd = a.shape[0] if trans_a else a.shape[1]
        fusable = (use_native(a) and not trans_a and not trans_b and bias is None
                   and act == "none" and c is None and (out_dtype in (None, a.dtype))
                   and M % 8 == 0 and N % 8 == 0 and Kd % 8 == 0
                   and addend.dtype == a.dtype and addend.is_contiguous())
        if fusable:
            return native().gemm(a, b, False, False, None, "none", a.dtype, None, 0.0, -1,
                                 addend.reshape(M, N), prefetch)
        return gemm(a, b, trans_a, trans_b, bias, act, out_dtype, c, beta) + addend.reshape(M, N)
    if use_native(a):
        odt = out_dtype if out_dtype is not None else a.dtype
        M = a.shape[1] if trans_a else a.shape[0]
        Kd = a.shape[0] if trans_a else a.shape[1]
        N = b.shape[0] if trans_b else b.shape[1]
        r8 = lambda v: (v + 7) // 8 * 8  # noqa: E731
        if M % 8 == 0 and N % 8 == 0 and Kd % 8 == 0:
            return native().gemm(a, b, trans_a, trans_b, bias, act, odt, c, beta, -1, None,
                                 prefetch)
        # odd sizes (e.g. a 10-class head): zero-pad every operand dim to a multiple of 8 —
        # the kernels vectorise 16-byte rows; the pad contributes exact zeros
        Mp, Np, Kp = r8(M), r8(N), r8(Kd)
        ap = _pad2(a, Kp, Mp) if trans_a else _pad2(a, Mp, Kp)
        bp = _pad2(b, Np, Kp) if trans_b else _pad2(b, Kp, Np)
        biasp = None
        if bias is not None:
            biasp = bias.new_zeros(Np)
            biasp[:N] = bias
        accumulate = c is not None and beta != 0.0
        y = native().gemm(ap.contiguous(), bp.contiguous(), trans_a, trans_b, biasp, act,
                          torch.float32 if accumulate else odt, None, 0.0)
        y = y[:M, :N]
        if accumulate:
            c.add_(y)
            return c
        return y.contiguous()
    return _ref.gemm(a, b, trans_a, trans_b, bias, act, out_dtype, c, beta)


def cross_entropy_fwd_bwd(logits, labels, label_smoothing=0.0, ignore_index=-100, valid_cols=-1):
    """``valid_cols``: only the first columns are classes (the rest pad a vocabulary to the GEMM
    tile width: excluded from the softmax, gradient 0)."""
    if use_native(logits):
        return native().cross_entropy_fwd_bwd(logits, labels, label_smoothing, ignore_index,
                                              valid_cols)
    return _ref.cross_entropy_fwd_bwd(logits, labels, label_smoothing, ignore_index, valid_cols)


def top1_correct(logits, labels, out=None):
    """``out`` (int32 [1], device) += number of rows whose argmax equals the label — the
    reference's eval accumulation (task.py:36-44) as one kernel, no host sync."""
    if use_native(logits):
        return native().top1_correct(logits.contiguous(), labels.contiguous(), out)
    n = (logits.argmax(1) == labels).sum().to(torch.int32).reshape(1)
    if out is None:
        return n
    out.add_(n)
    return out


def sgd_step(param, grad, mom, shadow, lr, momentum, dampening, weight_decay, nesterov,
             first_step, grad_scale=1.0):
    if use_native(param):
        return native().sgd_step(param, grad, mom, shadow, lr, momentum, dampening,
                                 weight_decay, nesterov, first_step, grad_scale)
    return _ref.sgd_step(param, grad, mom, shadow, lr, momentum, dampening, weight_decay,
                         nesterov, first_step, grad_scale)


def adamw_step(param, grad, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2, eps, weight_decay,
               step, grad_scale=1.0, step_dev=None):
    """``step_dev``: int32 [1] device step count; the kernel then computes the bias corrections
    itself (graph-replayable), ``step`` is ignored by the native path."""
    if use_native(param):
        return native().adamw_step(param, grad, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2,
                                   eps, weight_decay, step, grad_scale, step_dev)
    if step_dev is not None:
        step = int(step_dev.reshape(-1)[0].item())
    return _ref.adamw_step(param, grad, exp_avg, exp_avg_sq, shadow, lr, beta1, beta2, eps,
                           weight_decay, step, grad_scale)


def layernorm_fwd(x, gamma, beta, eps, residual=None, drop=None):
    """-> (y, mean, rstd, xsum).  ``drop=(p, seed)`` (needs ``residual``): y = LN(dropout(x) +
    residual), the dropout mask being :func:`dropout_fwd`'s for that seed."""
    if use_native(x):
        if drop is not None and drop[0] > 0.0:
            sd, dev = _split_seed(drop[1])
            return native().layernorm_fwd(x, gamma, beta, eps, residual, drop[0], sd, dev)
        return native().layernorm_fwd(x, gamma, beta, eps, residual)
    if drop is not None and drop[0] > 0.0:
        x = dropout_fwd(x, drop[0], drop[1])
    return _ref.layernorm_fwd(x, gamma, beta, eps, residual)


def layernorm_bwd(dy, x, mean, rstd, gamma, acc=None, drop=None, dbias=None):
    """-> (dx, dgamma, dbeta, dxd); with ``acc=(dgamma_buf, dbeta_buf)`` the parameter grads are
    accumulated into those buffers and returned as None.  ``drop=(p, seed)``: dxd = dropout'(dx),
    the gradient of the dropped branch (else None).  ``dbias`` (fp32 [H]): also += Σ_rows of the
    branch gradient (dxd, else dx) — the bias gradient of the Linear that produced x."""
    if use_native(dy):
        a = acc if acc is not None else (None, None)
        if drop is not None and drop[0] > 0.0:
            sd, dev = _split_seed(drop[1])
            return native().layernorm_bwd(dy, x, mean, rstd, gamma, *a, drop[0], sd, dev, dbias)
        return native().layernorm_bwd(dy, x, mean, rstd, gamma, *a, dbias=dbias)
    dx, dg, db = _ref.layernorm_bwd(dy, x, mean, rstd, gamma)
    dxd = dropout_fwd(dx, drop[0], drop[1]) if drop is not None and drop[0] > 0.0 else None
    if dbias is not None:
        colsum((dxd if dxd is not None else dx).reshape(-1, dx.shape[-1]), dbias)
    if acc is not None:
        acc[0].add_(dg.to(acc[0].dtype))
        acc[1].add_(db.to(acc[1].dtype))
        return dx, None, None, dxd
    return dx, dg, db, dxd


def colsum(x, out=None):
    """Σ over rows of a [rows, cols] tensor in fp32; accumulates into ``out`` when given."""
    if use_native(x) and x.shape[-1] % 8 == 0 and x.dtype in (torch.bfloat16, torch.float32):
        return native().colsum(x.contiguous(), out)
    s = x.reshape(-1, x.shape[-1]).to(torch.float64 if x.dtype == torch.float64 else torch.float32).sum(0)
    if out is not None:
        out.add_(s.to(out.dtype))
        return out
    return s


class DevSeed(NamedTuple):
    """A dropout seed whose per-step part lives on the device: ``base`` (host, per call site)
    mixed inside the kernel with ``counter`` (int32 [1] device tensor advanced once per training
    step by a device op).  A replayed hipGraph therefore draws a fresh mask every step."""
    base: int
    counter: torch.Tensor


def _split_seed(seed):
    """(host seed, device counter or None) for the native kernels."""
    if isinstance(seed, DevSeed):
        return seed.base & 0xFFFFFFFF, seed.counter
    return int(seed) & 0xFFFFFFFF, None


def _host_seed(seed) -> int:
    """The plain-torch reference path: fold the counter value in on the host (no graphs there)."""
    if isinstance(seed, DevSeed):
        c = int(seed.counter.reshape(-1)[0].item())
        return (seed.base ^ (c * 0x9E3779B1 + 0x632BE5AB)) & 0xFFFFFFFF
    return int(seed)


def attention_fwd(qkv, B, S, H, mask, scale, p_drop=0.0, seed=0):
    if use_native(qkv):
        sd, dev = _split_seed(seed)
        return native().attention_fwd(qkv, B, S, H, mask, scale, p_drop, sd, dev)
    return _ref.attention_fwd(qkv, B, S, H, mask, scale, p_drop, _host_seed(seed))


def attention_bwd(do, qkv, o, lse, B, S, H, mask, scale, p_drop=0.0, seed=0):
    if use_native(do):
        sd, dev = _split_seed(seed)
        return native().attention_bwd(do, qkv, o, lse, B, S, H, mask, scale, p_drop, sd, dev)
    return _ref.attention_bwd(do, qkv, o, lse, B, S, H, mask, scale, p_drop, _host_seed(seed))


def dropout_fwd(x, p, seed):
    """y = x·keep/(1-p) with keep hashed from (seed, element index); applying it to dy with the
    same seed is the backward.  ``seed``: int or :class:`DevSeed`."""
    if use_native(x) and x.numel() % 8 == 0:
        sd, dev = _split_seed(seed)
        return native().dropout_fwd(x, p, sd, dev)
    return _ref.dropout_fwd(x, p, _host_seed(seed))


def embedding_bwd(dy, idx, num_rows, out=None, ordered: bool = False, scale: float = 1.0,
                  presorted=None):
    """Scatter-add of ``scale`` * dy rows into a [num_rows, H] fp32 table gradient (``out``:
    accumulate into it, e.g. the parameter's flat-gradient view; else a fresh zeroed tensor).
    ``ordered`` (implied in deterministic mode): no float atomics — rows are summed per table row
    in token order (stable sort of the ids), so the result is bit-reproducible.  ``presorted``:
    (sorted ids, positions) of a stable sort of ``idx`` computed ahead (implies ordered); ids may
    then be negative — padding rows, skipped."""
    if use_native(dy):
        sid, perm = presorted if presorted is not None else (None, None)
        return native().embedding_bwd(dy, idx, num_rows, out, bool(ordered), float(scale),
                                      sid, perm)
    if presorted is not None or bool((idx < 0).any()):
        keep = idx.reshape(-1) >= 0
        dy = dy.reshape(-1, dy.shape[-1])[keep]
        idx = idx.reshape(-1)[keep]
    g = _ref.embedding_bwd(dy, idx, num_rows)
    if scale != 1.0:
        g = g * scale
    if out is not None:
        out.add_(g.to(out.dtype))
        return out
    return g


def gelu_fwd(x):
    if use_native(x):
        return native().gelu_fwd(x)
    return _ref.gelu_fwd(x)


def gelu_bwd(dy, x):
    if use_native(dy):
        return native().gelu_bwd(dy, x)
    return _ref.gelu_bwd(dy, x)


def gelu_bwd_colsum_ok(dy) -> bool:
    """gelu_bwd_colsum runs as one native kernel for this [rows, cols] bf16 gradient."""
    return use_native(dy) and dy.dtype == torch.bfloat16 and dy.shape[-1] % 8 == 0


def gelu_bwd_colsum(dy, x, bias):
    """dx = gelu_bwd(dy, x), and bias (fp32 [cols]) += Σ_rows dx — the bf16-rounded dx, so the
    result equals colsum(gelu_bwd(dy, x), bias) bit for bit (same per-column summation order)."""
    if gelu_bwd_colsum_ok(dy):
        return native().gelu_bwd_colsum(dy.contiguous(), x.contiguous(), bias)
    dx = gelu_bwd(dy, x)
    colsum(dx.reshape(-1, dx.shape[-1]), bias)
    return dx


def stem_pack(x, dtype, pad: int, Hp: int, Wsp: int, w=None):
    """NCHW image (C <= 4) -> bf16/``dtype`` super-pixels [N, Hp, Wsp, 8]: channel p*4 + c of
    super-pixel (h', j) is x[c, h'-pad, 2j+p-pad] (zero outside the image).  ``w`` (native, fp32
    [Co, C, K, K]): the same launch also packs the filter -> returns (x_packed, w_packed
    [Co, K, ceil(K/2), 8]) with w_packed[co][kh][j][p*4 + c] = w[co][c][kh][2j + p]."""
    if use_native(x) and dtype in (torch.bfloat16, torch.float32):
        y, wp = native().stem_pack(x.contiguous(), pad, Hp, Wsp, dtype, w)
        return (y, wp) if w is not None else y
    if w is not None:
        raise RuntimeError("stem_pack with the filter is a native-kernel path")
    N, C, H, W = x.shape
    P = x.new_zeros(N, 4, Hp, 2 * Wsp, dtype=torch.float64 if x.dtype == torch.float64 else torch.float32)
    hh, ww = min(H, Hp - pad), min(W, 2 * Wsp - pad)
    P[:, :C, pad:pad + hh, pad:pad + ww] = x[:, :, :hh, :ww].to(P.dtype)
    y = P.reshape(N, 4, Hp, Wsp, 2).permute(0, 2, 3, 4, 1).reshape(N, Hp, Wsp, 8)
    return y.contiguous().to(dtype)


# ----------------------------------------------------------------------------- vision.hip
_ACT = {"none": 0, "relu": 1, "relu6": 2}


def gconv_fwd(x, w, stride, pad, groups, bias=None, act="none"):
    """Direct NHWC convolution for grouped / depthwise / non-square / odd-channel convs:
    y = act(conv(x, w) + bias), w [Co, KH, KW, Ci/groups]; ``stride`` / ``pad`` are (h, w)."""
    if use_native(x):
        return native().gconv_fwd(x, w, list(stride), list(pad), int(groups), bias, _ACT[act])
    return _ref.gconv_fwd(x, w, stride, pad, groups, bias, act)


def gconv_dgrad(dy, w, x_shape, stride, pad, groups, z=None, act="none"):
    """dx.  ``z``: the forward output when an activation was fused (dy masked by act'(z))."""
    if use_native(dy):
        return native().gconv_dgrad(dy, w, list(x_shape), list(stride), list(pad), int(groups),
                                    z, _ACT[act])
    return _ref.gconv_dgrad(dy, w, x_shape, stride, pad, groups, z, act)


def gconv_wgrad(dy, x, kh, kw, stride, pad, groups, z=None, act="none", out=None, dbias=None,
                want_bias=False):
    """(dw [Co, KH, KW, Ci/groups] fp32, db [Co] fp32 | None).  ``out`` / ``dbias``: accumulate
    into these (flat-gradient views) instead of fresh buffers."""
    if use_native(dy):
        return native().gconv_wgrad(dy, x, kh, kw, list(stride), list(pad), int(groups), z,
                                    _ACT[act], out, dbias, bool(want_bias))
    dw, db = _ref.gconv_wgrad(dy, x, kh, kw, stride, pad, groups, z, act)
    if out is not None:
        out.add_(dw)
        dw = out
    if dbias is not None:
        dbias.add_(db)
        db = dbias
    return dw, (db if (want_bias or dbias is not None) else None)


def chan_stats(y, shift):
    """Shifted per-channel Σ(y - shift), Σ(y - shift)² of an NHWC tensor ([1, C] fp32 each)."""
    if use_native(y):
        return native().chan_stats(y, shift)
    return _ref.chan_stats(y, shift)


def affine_act(y, scale, bias, act="none"):
    """act(y * scale + bias) per channel (BatchNorm apply for any channel count)."""
    if use_native(y):
        return native().affine_act(y, scale, bias, _ACT[act])
    return _ref.affine_act(y, scale, bias, act)


def bn_generic_bwd_reduce(dz, z, y, mean, invstd, act="none"):
    if use_native(dz):
        return native().bn_generic_bwd_reduce(dz, z, y, mean, invstd, _ACT[act])
    return _ref.bn_generic_bwd_reduce(dz, z, y, mean, invstd, act)


def bn_generic_bwd_apply(dz, z, y, mean, invstd, gamma, sum_g, sum_gx, count, act="none"):
    if use_native(dz):
        return native().bn_generic_bwd_apply(dz, z, y, mean, invstd, gamma, sum_g, sum_gx,
                                             int(count), _ACT[act])
    return _ref.bn_generic_bwd_apply(dz, z, y, mean, invstd, gamma, sum_g, sum_gx, count, act)


def avgpool2d_fwd(x, k, stride, pad):
    if use_native(x):
        return native().avgpool2d_fwd(x, k, stride, pad)
    return _ref.avgpool2d_fwd(x, k, stride, pad)


def avgpool2d_bwd(dy, x_shape, k, stride, pad):
    if use_native(dy):
        return native().avgpool2d_bwd(dy, list(x_shape), k, stride, pad)
    return _ref.avgpool2d_bwd(dy, x_shape, k, stride, pad)


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
