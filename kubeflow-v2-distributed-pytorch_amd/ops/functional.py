"""Autograd functions over the fused kernel contracts (see :mod:`mipipe.ops.kernels`).

The training step of the reference (task.py:308-312: zero_grad, forward, CE loss,
backward, SGD step) decomposes into these units, each one or two HIP launches:

* :func:`conv2d` — implicit-GEMM convolution (MFMA) whose epilogue also emits the
  per-channel partial sums BatchNorm needs, so BN never re-reads the conv output for stats;
* :func:`batchnorm_act` — BN normalize/affine + optional residual add (raw identity or a
  second BN'd branch) + ReLU in one pass; backward = one reduce pass + one apply pass that
  also produces the residual gradient;
* :func:`linear`, :func:`cross_entropy`, :func:`max_pool2d`, :func:`global_avg_pool`,
  :func:`layer_norm`, :func:`gelu`, :func:`attention`, :func:`embedding`.

Master weights stay fp32 (``nn.Parameter``); kernels consume a compute-dtype *shadow*
(bf16 on the GPU) passed as a separate, non-differentiable argument; weight gradients come
back in fp32.
"""
from __future__ import annotations

import math
import os
import weakref
from dataclasses import dataclass
from typing import Optional, Tuple

import torch
from torch.autograd import Function

from . import kernels as K
from . import prefetch as _prefetch

Tensor = torch.Tensor


# block-output ReLU masks kept as bits for the fused backward (MIPIPE_RELU_BITMASK=0: read z)
_RELU_BITMASK = os.environ.get("MIPIPE_RELU_BITMASK", "1") != "0"

# Weight-grads on a side stream (MIPIPE_SIDE_WGRAD=1): a conv's weight-grad is off the backward
# critical path (dgrad -> BN apply -> next dgrad), so it can run beside the chain; the side
# stream joins the compute stream at the end of backward (engine callback).
_SIDE_WGRAD = os.environ.get("MIPIPE_SIDE_WGRAD", "0") == "1"
_SIDE_STREAMS = {}
_SIDE_JOIN_PENDING = set()


def _side_stream(t: Tensor):
    key = t.device.index
    s = _SIDE_STREAMS.get(key)
    if s is None:
        s = torch.cuda.Stream(t.device)
        _SIDE_STREAMS[key] = s
    return s


def _queue_side_join(main, side) -> None:
    key = id(side)
    if key in _SIDE_JOIN_PENDING:
        return
    _SIDE_JOIN_PENDING.add(key)

    def join():
        _SIDE_JOIN_PENDING.discard(key)
        main.wait_stream(side)
    torch.autograd.Variable._execution_engine.queue_callback(join)


# ----------------------------------------------------------------------------- conv
def _direct_grad_target(p: Tensor, rows: Optional[int] = None):
    """If ``p.grad`` is p's view in a flat gradient buffer, return (space, grad) so a kernel can
    accumulate straight into it (the DDP bucket), else None.  ``rows``: the caller computes a
    gradient with dim 0 padded to ``rows`` (a tile-padded vocabulary); the target is then the
    space's padded view (the pad rows are reserved zeros in the flat buffers), or None."""
    from mipipe.optim.flat import flat_space_for
    if not p.is_leaf:
        return None
    fs = flat_space_for(p)
    g = p.grad
    if fs is None or g is None or not g.is_cuda:
        return None
    if g.data_ptr() != fs.flat_grad.data_ptr() + 4 * fs.offset(p):
        return None
    if rows is not None and rows != p.shape[0]:
        if fs.padded_rows(p) != rows:
            return None
        return fs, fs.padded_view(fs.flat_grad, p)
    return fs, g


def _wgrad_map_into_grad(wmap, dw, weight):
    """A kernel-layout weight gradient (packed stem filter) for ``weight``: accumulated straight
    into its flat-buffer gradient by one native launch when the map supports it (returns None:
    nothing left for autograd to add), else mapped to the parameter layout and returned."""
    acc = getattr(wmap, "accumulate_into", None)
    tgt = _direct_grad_target(weight) if acc is not None else None
    if tgt is not None and acc(dw, tgt[1]):
        tgt[0].grad_ready(weight)
        return None
    return wmap(dw).to(weight.dtype)


class ResidualSlot:
    """Hands a block input's second gradient (identity / downsample path) to the conv that
    also consumes that input, so its dgrad epilogue adds it (no separate elementwise add).

    Order-independent: a producer that runs before the consumer stashes its gradient and
    returns None to autograd; if the consumer already ran, the producer returns it normally."""

    __slots__ = ("pending", "consumed")

    def __init__(self):
        self.pending = None
        self.consumed = False

    def produce(self, g):
        if g is None or self.consumed:
            return g
        self.pending = g if self.pending is None else self.pending + g
        return None

    def take(self):
        self.consumed = True
        p, self.pending = self.pending, None
        return p


class BiasGradSlot:
    """Links a Linear to the LayerNorm that consumes its output (BERT's post-LN branches): the
    LayerNorm backward, which writes the branch gradient anyway, also sums it over rows into the
    Linear bias's flat-gradient view, and the Linear's backward skips its column-sum pass."""

    __slots__ = ("bias", "done")

    def __init__(self):
        self.bias = None
        self.done = False


class BNActToken:
    """Links a BN(+ReLU) output to its single consuming conv: the conv's backward computes the
    BN-backward reductions in its dgrad epilogue and flags the BN's backward to skip them."""

    __slots__ = ("bn", "st", "y", "_z", "mask", "pre_reduced", "collected", "y2", "st2", "bn2",
                 "rep")

    @property
    def z(self):
        return None if self._z is None else self._z()

    @z.setter
    def z(self, t):
        # weak: z carries this token as ``z._mipipe_bnact``; a strong back-reference would make
        # a z <-> token cycle that holds every block output until the next gc pass
        self._z = None if t is None else weakref.ref(t)

    def __init__(self, bn, st, y, z=None):
        # z set: BN + residual + ReLU block output.  Its consumer conv also feeds the next
        # block's identity path, so the fusion is valid only when that conv's dgrad also adds
        # the identity gradient (residual slot delivered) - the mask comes from stored z, or
        # from its 1-bit copy (``mask``, written by the BN-apply kernel: 1/16 of z's bytes).
        self.bn, self.st, self.y, self.z = bn, st, y, z
        self.mask = None
        self.pre_reduced = False
        # (Σg/Σg·x̂[/Σg·x̂₂] [2|3, C], direct dγ/dβ accumulated, direct dγ₂/dβ₂ accumulated) when
        # the consuming conv's weight-grad launch already collected the bwd slab (BnCollect)
        self.collected = None
        # two-branch block output relu(bn(y) + bn2(y2)) (ResNet downsample block)
        self.y2 = self.st2 = self.bn2 = None
        self.rep = None  # the bwd slab the consuming dgrad filled (this pass's own slab)


_TAP_CROP = os.environ.get("MIPIPE_TAP_CROP", "1") != "0"
_CONV_FLATTEN = os.environ.get("MIPIPE_CONV_FLATTEN", "1") != "0"


def tap_crop(x_shape, w_shape, stride, pad):
    """Filter taps that can never touch the image for this geometry are dropped (the analogue
    of cuDNN picking an algorithm per shape): a 3x3 / pad-1 conv on a 1x1 feature map (ResNet-18
    layer 4 at 32x32, the reference's config of record) only ever reads its centre tap — a 1x1
    GEMM with K = Ci instead of 9 Ci, 8/9 of the MFMA work spent on padding otherwise.

    Returns (kh0, kh1, kw0, kw1, pad') — the kept tap ranges and the padding that maps every
    output to the same input pixels — or None when every tap is used somewhere, the output size
    would change, or the cropped padding is not square."""
    if not (_TAP_CROP and isinstance(stride, int) and isinstance(pad, int)):
        return None
    _, H, W, _ = x_shape
    _, KH, KW, _ = w_shape
    Ho, Wo = (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1

    def span(L, Lo, K):
        used = [k for k in range(K) if any(0 <= o * stride - pad + k < L for o in range(Lo))]
        return (used[0], used[-1] + 1) if used else (0, K)
    (h0, h1), (w0, w1) = span(H, Ho, KH), span(W, Wo, KW)
    if (h0, h1, w0, w1) == (0, KH, 0, KW) or pad - h0 != pad - w0:
        return None
    p2 = pad - h0
    if ((H + 2 * p2 - (h1 - h0)) // stride + 1 != Ho
            or (W + 2 * p2 - (w1 - w0)) // stride + 1 != Wo):
        return None
    return h0, h1, w0, w1, p2


class _ConvFn(Function):
    @staticmethod
    def forward(ctx, x, weight, w_c, stride, pad, shift, slabs=None, prev=None, res_take=None,
                res_give=None, in_bn=None):
        # in_bn = (scale, bias): x holds y of a BatchNorm + ReLU folded into this conv (dense 1x1,
        # see conv_bn_act(fold_next=)): the forward and the weight-grad transform their operand
        ctx.in_bn = in_bn
        # taps that never touch the image are cropped away (forward, data-grad and weight-grad
        # all run the smaller filter; the weight-grad lands in its slice of the full gradient)
        crop = (tap_crop(tuple(x.shape), tuple(w_c.shape), stride, pad)
                if getattr(weight, "_mipipe_wgrad_map", None) is None and in_bn is None else None)
        if crop is not None:
            kh0, kh1, kw0, kw1, pad = crop
            w_c = w_c[:, kh0:kh1, kw0:kw1, :].contiguous()
        ctx.full_k = (weight.shape[2], weight.shape[3])
        # a (cropped) filter that covers the whole unpadded input has ONE output pixel: the conv
        # is a 1x1 conv of the flattened image ([N, 1, 1, H*W*C] x [Co, 1, 1, KH*KW*C], the NHWC
        # and [Co, KH, KW, Ci] orders agree) — one dense GEMM for the data-grad instead of a launch
        # per stride-parity class (ResNet-18 layer 4's stride-2 conv on its 2x2 map)
        ctx.flat = None
        if (_TAP_CROP and _CONV_FLATTEN and isinstance(stride, int) and isinstance(pad, int)
                and pad == 0 and in_bn is None
                and getattr(weight, "_mipipe_wgrad_map", None) is None
                and w_c.shape[1] == x.shape[1] and w_c.shape[2] == x.shape[2]
                and w_c.shape[3] == x.shape[3] and x.shape[1] * x.shape[2] > 1):
            if crop is None:
                crop = (0, w_c.shape[1], 0, w_c.shape[2], 0)
            ctx.flat = tuple(x.shape)
            n, h, w_, c = x.shape
            x = x.reshape(n, 1, 1, h * w_ * c)
            w_c = w_c.reshape(w_c.shape[0], 1, 1, h * w_ * c)
            stride = 1
        ctx.crop = crop
        # stride-1 k x k convs: the forward launch also writes the tap-flipped weight the
        # data-grad reads (a persistent buffer per weight; no flip kernel in the backward)
        wflip = None
        if (x.requires_grad and K.use_native(x) and isinstance(stride, int)
                and isinstance(pad, int) and K.dgrad_preflip_ok(x.shape, w_c.shape, stride, pad)):
            wflip = weight.__dict__.get("_mipipe_wflip")
            if (wflip is None or wflip.numel() != w_c.numel() or wflip.dtype != w_c.dtype
                    or wflip.device != w_c.device):
                wflip = torch.empty(w_c.numel(), dtype=w_c.dtype, device=w_c.device)
                weight.__dict__["_mipipe_wflip"] = wflip
        y, psum, psumsq = K.conv_fwd(x, w_c, stride, pad, shift, slabs, wflip=wflip, in_bn=in_bn)
        ctx.wflip = wflip
        ctx.set_materialize_grads(False)  # stats outputs never get gradients: no zero fills
        ctx.save_for_backward(x, w_c)
        ctx.weight = weight
        # kernel-layout weight dims (the packed stem differs from the parameter's)
        ctx.conf = (stride, pad, w_c.shape[1], w_c.shape[2], weight.shape[1])
        ctx.wmap = getattr(weight, "_mipipe_wgrad_map", None)
        ctx.prev, ctx.res_take, ctx.res_give = prev, res_take, res_give
        if psum is not None:
            ctx.mark_non_differentiable(psum, psumsq)
        return y, psum, psumsq

    @staticmethod
    def backward(ctx, dy, _g1, _g2):
        x, w_c = ctx.saved_tensors
        if dy is None:
            return (None,) * 11
        in_bn = ctx.in_bn
        stride, pad, kh, kw, ci = ctx.conf
        dy = dy.contiguous()
        dx = dw = None
        bnr = tok = None
        if ctx.needs_input_grad[0]:
            if not isinstance(stride, int):
                raise NotImplementedError("dgrad of a non-square-stride conv")
            addend = ctx.res_take.take() if ctx.res_take is not None else None
            bnr = None
            tok = ctx.prev if ctx.flat is None else None  # flattened: per-channel BN fusion off
            if ctx.flat is not None and addend is not None:
                addend = addend.reshape(x.shape)
            two = tok is not None and tok.y2 is not None
            # the two-branch fusion: bf16 1x1 stride-1 data-grads whose weight-grad launch (which
            # collects the third slab array) follows
            two_ok = (not two or (kh == 1 and kw == 1 and stride == 1 and pad == 0
                                  and dy.dtype == torch.bfloat16 and ctx.needs_input_grad[1]
                                  and tok.st2.batch_stats))
            if (tok is not None and K.use_native(dy) and tok.st.batch_stats and two_ok
                    and (tok.z is None or addend is not None)):
                rep = bn_workspace(tok.bn, "bwd", dy.device)  # zeroed; pending until collect
                tok.rep = rep
                if rep is not None:
                    st = tok.st
                    bnr = (tok.y, st.mean, st.invstd, st.scale, st.bias, rep)
                    if tok.z is not None:
                        bnr = bnr + (tok.mask if tok.mask is not None else tok.z,)
            bnr2 = (tok.y2, tok.st2.mean, tok.st2.invstd) if bnr is not None and two else None
            dx = K.conv_dgrad(dy, w_c, x.shape, stride, pad, addend=addend, bnr=bnr, bnr2=bnr2,
                              wflip=ctx.wflip)
            if bnr is not None:
                tok.pre_reduced = True
            if ctx.flat is not None:
                dx = dx.reshape(ctx.flat)
            if ctx.res_give is not None:
                dx = ctx.res_give.produce(dx)
        if ctx.needs_input_grad[1]:
            weight = ctx.weight
            collect = None
            cin = x.shape[-1] if ctx.flat is None else ctx.flat[-1]
            tgt = (_direct_grad_target(weight)
                   if cin == ci and ctx.wmap is None and K.use_native(dy) else None)
            side = None
            if (_SIDE_WGRAD and tgt is not None and dy.is_cuda and not tgt[0]._ready_listeners
                    and not (bnr is not None and tok.y2 is not None) and ctx.crop is None):
                side = _side_stream(dy)
            if bnr is not None and side is None:
                # the weight-grad launch also collects the slab the fused dgrad just filled
                # (one of its blocks; no separate bn_bwd_collect launch)
                two = tok.y2 is not None
                bn = tok.bn
                out2 = torch.empty(3 if two else 2, bn.num_features, device=dy.device,
                                   dtype=torch.float32)

                def targets(m):
                    tg = _direct_grad_target(m.weight) if m.weight is not None else None
                    tb = _direct_grad_target(m.bias) if m.bias is not None else None
                    ok = (tg is not None and tb is not None and m.weight.requires_grad
                          and m.bias.requires_grad)
                    return (tg[1], tb[1]) if ok else (None, None)
                t1 = targets(bn)
                t2 = targets(tok.bn2) if two else (None, None)
                collect = (bnr[5], out2) + t1 + ((True,) + t2 if two else ())
                tok.collected = (out2, t1[0] is not None, t2[0] is not None)
            if side is not None:
                # the BN backward collects its own slab (bn_bwd_collect) on the compute stream
                fs, g = tgt
                main = torch.cuda.current_stream(dy.device)
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    K.conv_wgrad(dy, x, kh, kw, stride, pad, out=g.permute(0, 2, 3, 1),
                                 in_bn=in_bn)
                dy.record_stream(side)
                x.record_stream(side)
                _queue_side_join(main, side)
                fs.grad_ready(weight)
            elif tgt is not None:
                # gradient accumulates straight into the flat DDP bucket: no zero-fill, no
                # autograd AccumulateGrad add; tell the reducer the gradient is ready.
                fs, g = tgt
                if ctx.crop is not None:  # the kept taps' slice of the full gradient
                    kh0, kh1, kw0, kw1, _ = ctx.crop
                    part = K.conv_wgrad(dy, x, kh, kw, stride, pad, collect=collect)
                    g.permute(0, 2, 3, 1)[:, kh0:kh1, kw0:kw1, :].add_(
                        part.reshape(part.shape[0], kh1 - kh0, kw1 - kw0, -1))
                else:
                    K.conv_wgrad(dy, x, kh, kw, stride, pad, out=g.permute(0, 2, 3, 1),
                                 collect=collect, in_bn=in_bn)
                fs.grad_ready(weight)
            else:
                dw = K.conv_wgrad(dy, x, kh, kw, stride, pad, collect=collect, in_bn=in_bn)
                if ctx.crop is not None:
                    kh0, kh1, kw0, kw1, _ = ctx.crop
                    dw = dw.reshape(dw.shape[0], kh1 - kh0, kw1 - kw0, -1)
                    full = dw.new_zeros(dw.shape[0], ctx.full_k[0], ctx.full_k[1], dw.shape[3])
                    full[:, kh0:kh1, kw0:kw1, :] = dw
                    dw = full
                if ctx.wmap is not None:  # kernel layout -> parameter layout (packed stem)
                    dw = _wgrad_map_into_grad(ctx.wmap, dw, weight)
                else:
                    if dw.shape[-1] != ci:  # input channels were zero-padded for the kernel
                        dw = dw[..., :ci]
                    dw = dw.permute(0, 3, 1, 2)
        return dx, dw, None, None, None, None, None, None, None, None, None


def conv2d(x: Tensor, weight: Tensor, w_c: Tensor, stride: int, pad: int,
           stats_shift: Optional[Tensor] = None, slabs=None, prev: Optional[BNActToken] = None,
           res_take: Optional[ResidualSlot] = None, res_give: Optional[ResidualSlot] = None,
           in_bn=None):
    """NHWC conv.  Returns (y, psum, psumsq); the partials are None unless ``stats_shift``.
    ``prev``: token of the BN(+ReLU) that produced x (x has no other consumer) -> BN-backward
    reductions fused into this conv's dgrad.  ``res_take`` / ``res_give``: residual-gradient
    slot this conv's dgrad adds / hands over (see :class:`ResidualSlot`).  ``in_bn = (scale,
    bias)``: x holds y of a BatchNorm + ReLU folded into this conv (bf16 dense 1x1)."""
    return _ConvFn.apply(x, weight, w_c, stride, pad, stats_shift, slabs, prev, res_take,
                         res_give, in_bn)


class _ConvBiasActFn(Function):
    """y = act(conv(x) + b) with bias and ReLU in the conv epilogue (VGG / AlexNet convs)."""

    @staticmethod
    def forward(ctx, x, weight, w_c, bias, stride, pad, relu):
        y, _, _ = K.conv_fwd(x, w_c, stride, pad, None, None, bias, relu)
        ctx.save_for_backward(x, w_c, y if relu else None)
        ctx.weight, ctx.bias = weight, bias
        ctx.conf = (stride, pad, weight.shape[2], weight.shape[3], weight.shape[1], relu)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_c, y = ctx.saved_tensors
        stride, pad, kh, kw, ci, relu = ctx.conf
        g = dy.contiguous()
        if relu:
            g = (g * (y > 0)).to(g.dtype)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = K.conv_dgrad(g, w_c, x.shape, stride, pad)
        native = K.use_native(g)
        if ctx.needs_input_grad[1]:
            tgt = _direct_grad_target(ctx.weight) if x.shape[-1] == ci and native else None
            if tgt is not None:
                K.conv_wgrad(g, x, kh, kw, stride, pad, out=tgt[1].permute(0, 2, 3, 1))
                tgt[0].grad_ready(ctx.weight)
            else:
                dw = K.conv_wgrad(g, x, kh, kw, stride, pad)
                if dw.shape[-1] != ci:
                    dw = dw[..., :ci]
                dw = dw.permute(0, 3, 1, 2)
        if ctx.bias is not None and ctx.needs_input_grad[3]:
            tb = _direct_grad_target(ctx.bias) if native else None
            if tb is not None:
                K.colsum(g.reshape(-1, g.shape[-1]), tb[1])
                tb[0].grad_ready(ctx.bias)
            else:
                db = K.colsum(g.reshape(-1, g.shape[-1])).to(ctx.bias.dtype)
        return dx, dw, None, db, None, None, None


def conv2d_bias_act(x: Tensor, weight: Tensor, w_c: Tensor, bias: Optional[Tensor], stride: int,
                    pad: int, relu: bool) -> Tensor:
    return _ConvBiasActFn.apply(x, weight, w_c, bias, stride, pad, relu)


class _GConvFn(Function):
    """Grouped / depthwise / non-square / odd-channel convolution (+bias, +activation) on the
    direct NHWC kernels of vision.hip.  The activation's mask is recomputed from the saved
    output in the backward kernels; weight (and bias) gradients accumulate straight into the
    flat DDP gradient buffer when the parameter lives there."""

    @staticmethod
    def forward(ctx, x, weight, w_c, bias, stride, pad, groups, act):
        y = K.gconv_fwd(x, w_c, stride, pad, groups, None if bias is None else bias.detach(), act)
        ctx.save_for_backward(x, w_c, y if act != "none" else None)
        ctx.weight, ctx.bias = weight, bias
        ctx.conf = (stride, pad, groups, act)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w_c, z = ctx.saved_tensors
        stride, pad, groups, act = ctx.conf
        weight, bias = ctx.weight, ctx.bias
        dy = dy.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = K.gconv_dgrad(dy, w_c, x.shape, stride, pad, groups, z, act)
        need_w = ctx.needs_input_grad[1]
        need_b = bias is not None and ctx.needs_input_grad[3]
        if need_w or need_b:
            native = K.use_native(dy)
            ci = weight.shape[1]
            padded = w_c.shape[-1] != ci  # input channels zero-padded for the kernel (stem)
            tw = _direct_grad_target(weight) if native and need_w and not padded else None
            tb = _direct_grad_target(bias) if native and need_b else None
            g_w, g_b = K.gconv_wgrad(dy, x, w_c.shape[1], w_c.shape[2], stride, pad, groups, z,
                                     act, out=None if tw is None else tw[1].permute(0, 2, 3, 1),
                                     dbias=None if tb is None else tb[1], want_bias=need_b)
            if tw is not None:
                tw[0].grad_ready(weight)
            elif need_w:
                dw = (g_w[..., :ci] if padded else g_w).permute(0, 3, 1, 2).to(weight.dtype)
            if tb is not None:
                tb[0].grad_ready(bias)
            elif need_b:
                db = g_b.to(bias.dtype)
        return dx, dw, None, db, None, None, None, None


class _BlockGroupConvFn(Function):
    """Grouped convolution on the MFMA implicit-GEMM kernels: ``gb`` groups at a time form one
    dense conv with a block-diagonal weight (channel blocks of gb*Cig inputs / gb*Cog outputs,
    64 wide), so ResNeXt's 4..32-channel groups run on matrix cores instead of a scalar direct
    kernel.  The off-diagonal zeros cost gb x the grouped FLOPs at MFMA rate; wgrad keeps only
    the diagonal blocks of the dense weight gradient."""

    @staticmethod
    def forward(ctx, x, weight, w_c, stride, pad, groups, gb):
        Co, kh, kw, cig = w_c.shape
        cog = Co // groups
        nb = groups // gb
        eye = torch.eye(gb, dtype=w_c.dtype, device=w_c.device)
        wbd = (w_c.view(nb, gb, cog, kh, kw, 1, cig) * eye.view(1, gb, 1, 1, 1, gb, 1))
        wbd = wbd.reshape(nb, gb * cog, kh, kw, gb * cig)
        bi, bo = gb * cig, gb * cog
        ys = []
        for b in range(nb):
            xb = x if nb == 1 else x[..., b * bi:(b + 1) * bi].contiguous()
            ys.append(K.conv_fwd(xb, wbd[b].contiguous(), stride, pad)[0])
        ctx.save_for_backward(x, wbd)
        ctx.weight = weight
        ctx.conf = (stride, pad, groups, gb, kh, kw, cig, cog)
        return ys[0] if nb == 1 else torch.cat(ys, dim=-1)

    @staticmethod
    def backward(ctx, dy):
        x, wbd = ctx.saved_tensors
        stride, pad, groups, gb, kh, kw, cig, cog = ctx.conf
        nb = groups // gb
        bi, bo = gb * cig, gb * cog
        dy = dy.contiguous()
        dxs, dws = [], []
        for b in range(nb):
            xb = x if nb == 1 else x[..., b * bi:(b + 1) * bi].contiguous()
            dyb = dy if nb == 1 else dy[..., b * bo:(b + 1) * bo].contiguous()
            if ctx.needs_input_grad[0]:
                dxs.append(K.conv_dgrad(dyb, wbd[b].contiguous(), xb.shape, stride, pad))
            if ctx.needs_input_grad[1]:
                dwb = K.conv_wgrad(dyb, xb, kh, kw, stride, pad)  # [bo, kh, kw, bi]
                d = torch.diagonal(dwb.view(gb, cog, kh, kw, gb, cig), dim1=0, dim2=4)
                dws.append(d.permute(4, 0, 1, 2, 3))  # [gb, cog, kh, kw, cig]
        dx = None if not dxs else (dxs[0] if nb == 1 else torch.cat(dxs, dim=-1))
        dw = None
        if dws:
            dw = torch.cat(dws, 0).reshape(groups * cog, kh, kw, cig).permute(0, 3, 1, 2)
            dw = dw.to(ctx.weight.dtype)
        return dx, dw, None, None, None, None, None


def grouped_conv_mfma_blocks(groups: int, cig: int, cog: int, width: int = 64) -> int:
    """Groups per block for the block-diagonal MFMA path (0: not applicable).  Depthwise convs
    (1 channel per group) stay on the vector direct kernels: a 64x waste is not worth it."""
    if groups == 1 or cig != cog or cig < 4 or cig % 4:
        return 0
    if cig >= width:
        return 1 if cig % 8 == 0 else 0
    gb = width // cig
    if width % cig or groups % gb or (gb * cig) % 8:
        return 0
    return gb


def block_group_conv2d(x: Tensor, weight: Tensor, w_c: Tensor, stride: int, pad, groups: int,
                       gb: int) -> Tensor:
    """Grouped NHWC convolution as block-diagonal dense convs on the MFMA kernels."""
    return _BlockGroupConvFn.apply(x, weight, w_c, stride, pad, int(groups), int(gb))


def gconv2d(x: Tensor, weight: Tensor, w_c: Tensor, bias: Optional[Tensor], stride, pad,
            groups: int, act: str = "none") -> Tensor:
    """NHWC convolution with ``groups`` and (h, w) stride / padding on the direct kernels;
    ``act`` in {none, relu, relu6} is applied in the same pass."""
    return _GConvFn.apply(x, weight, w_c, bias, tuple(int(v) for v in stride),
                          tuple(int(v) for v in pad), int(groups), act)


# ----------------------------------------------------------------------------- batchnorm
@dataclass
class BNStats:
    mean: Tensor
    invstd: Tensor
    scale: Tensor
    bias: Tensor
    count: int
    batch_stats: bool


def bn_workspace(bn, kind: str, device) -> Optional[Tensor]:
    """Persistent zero-initialised replica slab for BN statistics on the GPU ('fwd': [2,R,C],
    'bwd': [3,R,C]).  Kernels that accumulate into it are always followed by the kernel that
    reads AND re-zeroes it.  A per-module 'pending' flag marks a slab between those two kernels:
    if it is still set when the slab is requested again, either a step was interrupted or the
    module is used twice in one graph (a chunk loop, shared weights) and the two backward passes
    interleave — a FRESH slab then replaces the cached one (the in-flight user keeps its own),
    instead of re-zeroing a slab another pass is still accumulating into."""
    if device.type != "cuda" or not K.native_available():
        return None
    C = bn.num_features
    R = K.native().STAT_REPLICAS
    attr = "_mipipe_ws_" + kind
    ws = bn.__dict__.get(attr)
    rows = 2 if kind == "fwd" else 3
    if ws is None or ws.device != device or ws.numel() != rows * R * C:
        ws = torch.zeros(rows, R, C, device=device, dtype=torch.float32)
        bn.__dict__[attr] = ws
    pend = "_mipipe_pending_" + kind
    if bn.__dict__.get(pend):
        ws = torch.zeros_like(ws)
        bn.__dict__[attr] = ws
    bn.__dict__[pend] = True
    return ws


def _ws_done(bn, kind: str) -> None:
    bn.__dict__["_mipipe_pending_" + kind] = False


def bn_stats_from_partials(psum, psumsq, count, bn, training: bool) -> BNStats:
    """Finalize batch statistics (training) or use running statistics (eval)."""
    if training:
        mom = 0.1 if bn.momentum is None else bn.momentum
        mean, invstd, scale, bias = K.bn_finalize(
            psum, psumsq, count, bn.running_mean, bn.weight.detach(), bn.bias.detach(),
            bn.running_mean if bn.track_running_stats else None,
            bn.running_var if bn.track_running_stats else None, mom, bn.eps,
            bn.num_batches_tracked if bn.track_running_stats else None)
        _ws_done(bn, "fwd")
        return BNStats(mean, invstd, scale, bias, count, True)
    up = (lambda t: t) if bn.running_var.dtype == torch.float64 else (lambda t: t.float())
    invstd = torch.rsqrt(up(bn.running_var) + bn.eps)
    scale = up(bn.weight.detach()) * invstd
    bias = up(bn.bias.detach()) - up(bn.running_mean) * scale
    return BNStats(up(bn.running_mean), invstd, scale, bias, count, False)


class _BNActFn(Function):
    @staticmethod
    def forward(ctx, y, gamma, beta, residual, y2, gamma2, beta2, st, st2, relu, bn=None,
                token=None, res_give=None, lazy=False):
        ctx.lazy = lazy
        if lazy:
            # folded into the single consuming 1x1 conv (conv_bn_act(fold_next=)): that conv reads
            # y and applies relu(y*scale + bias) to its operand fragments; nothing is written here.
            # The returned alias of y carries the pending transform for the consumer.
            z = y.view_as(y)
            ctx.save_for_backward(y, None, y2, gamma, gamma2)
            ctx.st, ctx.st2, ctx.relu = st, st2, relu
            ctx.has_res = False
            ctx.bn = bn
            ctx.beta, ctx.beta2 = beta, beta2
            ctx.token, ctx.res_give = token, res_give
            return z
        mask = None
        if (_RELU_BITMASK and token is not None and relu
                and (residual is not None or y2 is not None) and K.use_native(y)):
            # block output: its fused backward reads the ReLU mask as bits, not z
            mask = torch.empty(y.numel() // 8, dtype=torch.uint8, device=y.device)
            token.mask = mask
        z = K.bn_act_fwd(y, st.scale, st.bias, relu,
                         residual if y2 is None else y2,
                         None if st2 is None else st2.scale, None if st2 is None else st2.bias,
                         mask=mask)
        ctx.save_for_backward(y, z, y2, gamma, gamma2)
        ctx.st, ctx.st2, ctx.relu = st, st2, relu
        ctx.has_res = residual is not None
        ctx.bn = bn
        ctx.beta, ctx.beta2 = beta, beta2
        ctx.token, ctx.res_give = token, res_give
        return z

    @staticmethod
    def backward(ctx, dz):
        y, z, y2, gamma, gamma2 = ctx.saved_tensors
        st, st2, relu = ctx.st, ctx.st2, ctx.relu
        dz = dz.contiguous()
        tok = ctx.token
        if tok is not None and tok.pre_reduced:
            return _BNActFn._backward_pre_reduced(ctx, dz, y, gamma, y2, gamma2) + (None,)
        if ctx.lazy:  # the consumer did not reduce (no fused dgrad ran): materialise z here
            z = K.bn_act_fwd(y, st.scale, st.bias, relu)
        rep = bn_workspace(ctx.bn, "bwd", dz.device) if ctx.bn is not None else None
        # BN affine grads accumulate straight into the flat gradient buffer when possible
        direct = None
        if rep is not None and st.batch_stats and ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            tg, tb = _direct_grad_target(gamma), _direct_grad_target(ctx.beta)
            ok = tg is not None and tb is not None
            t2g = t2b = None
            if y2 is not None:
                t2g, t2b = _direct_grad_target(gamma2), _direct_grad_target(ctx.beta2)
                ok = ok and t2g is not None and t2b is not None and st2.batch_stats
            if ok:
                direct = (tg[1], tb[1], None if t2g is None else t2g[1],
                          None if t2b is None else t2b[1])
        sg, sgx, sgx2 = K.bn_act_bwd_reduce(dz, z, y, st.mean, st.invstd, relu, y2,
                                            None if st2 is None else st2.mean,
                                            None if st2 is None else st2.invstd, rep, direct)
        if ctx.bn is not None:
            _ws_done(ctx.bn, "bwd")
        if direct is not None:
            fs = _direct_grad_target(gamma)[0]
            for p in (gamma, ctx.beta) + ((gamma2, ctx.beta2) if y2 is not None else ()):
                fs.grad_ready(p)
        if st.batch_stats and (st2 is None or st2.batch_stats):
            a_g, a_gx, a_gx2 = sg, sgx, sgx2
        else:
            zero = torch.zeros_like(sg)
            a_g, a_gx = (sg, sgx) if st.batch_stats else (zero, zero)
            a_gx2 = None
            if st2 is not None:
                a_gx2 = sgx2 if st2.batch_stats else zero
        dy, other = K.bn_act_bwd_apply(
            dz, z, y, st.mean, st.invstd, gamma.detach(), a_g, a_gx, st.count, relu,
            want_dres=ctx.has_res, y2=y2, mean2=None if st2 is None else st2.mean,
            invstd2=None if st2 is None else st2.invstd,
            gamma2=None if gamma2 is None else gamma2.detach(), sum_gx2=a_gx2)
        dres = other if ctx.has_res else None
        if dres is not None and ctx.res_give is not None:
            dres = ctx.res_give.produce(dres)
        dy2 = other if y2 is not None else None
        if direct is not None:
            return dy, None, None, dres, dy2, None, None, None, None, None, None, None, None, None
        dgamma2 = sgx2 if y2 is not None else None
        dbeta2 = sg if y2 is not None else None
        return (dy, sgx.to(gamma.dtype), sg.to(gamma.dtype), dres, dy2,
                None if dgamma2 is None else dgamma2.to(gamma2.dtype),
                None if dbeta2 is None else dbeta2.to(gamma2.dtype), None, None, None, None,
                None, None, None)

    @staticmethod
    def _backward_pre_reduced(ctx, g, y, gamma, y2=None, gamma2=None):
        """The consuming conv's dgrad already produced g = dz·relu'(z) and Σg, Σg·x̂ (and
        Σg·x̂₂ of a two-branch output) in the bwd replica slab: collect them (+ direct dγ/dβ)
        and apply, no reduction pass."""
        tok = ctx.token
        tok.pre_reduced = False
        st, bn = ctx.st, ctx.bn
        rep = tok.rep if tok.rep is not None else bn.__dict__["_mipipe_ws_bwd"]
        tok.rep = None
        C = y.shape[-1]
        direct = None
        if y2 is not None:  # two-branch: always collected by the weight-grad launch
            out3, d1, d2 = tok.collected
            tok.collected = None
            sg, sgx, sgx2 = out3[0], out3[1], out3[2]
            _ws_done(bn, "bwd")
            st2 = ctx.st2
            for used, (ga, be) in ((d1, (gamma, ctx.beta)), (d2, (gamma2, ctx.beta2))):
                if used:
                    fs = _direct_grad_target(ga)[0]
                    fs.grad_ready(ga)
                    fs.grad_ready(be)
            dy, dy2 = K.bn_act_bwd_apply(g, g, y, st.mean, st.invstd, gamma.detach(), sg, sgx,
                                         st.count, False, y2=y2, mean2=st2.mean,
                                         invstd2=st2.invstd, gamma2=gamma2.detach(),
                                         sum_gx2=sgx2)
            return (dy, None if d1 else sgx.to(gamma.dtype), None if d1 else sg.to(gamma.dtype),
                    None, dy2, None if d2 else sgx2.to(gamma2.dtype),
                    None if d2 else sg.to(gamma2.dtype), None, None, None, None, None, None)
        if tok.collected is not None:  # collected by the consuming conv's weight-grad launch
            out2, used_direct, _ = tok.collected
            tok.collected = None
            sg, sgx = out2[0], out2[1]
            direct = (True,) if used_direct else None
        else:
            if ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
                tg, tb = _direct_grad_target(gamma), _direct_grad_target(ctx.beta)
                if tg is not None and tb is not None:
                    direct = (tg[1], tb[1])
            sg, sgx = K.bn_bwd_collect(rep, C, direct)
        _ws_done(bn, "bwd")
        if direct is not None:
            fs = _direct_grad_target(gamma)[0]
            fs.grad_ready(gamma)
            fs.grad_ready(ctx.beta)
        dy, _ = K.bn_act_bwd_apply(g, g, y, st.mean, st.invstd, gamma.detach(), sg, sgx,
                                   st.count, False)
        dres = None
        if ctx.has_res:  # gradient of the pre-ReLU sum = g itself: hand it on, no copy
            dres = ctx.res_give.produce(g) if ctx.res_give is not None else g
        if direct is not None:
            return dy, None, None, dres, None, None, None, None, None, None, None, None, None
        return (dy, sgx.to(gamma.dtype), sg.to(gamma.dtype), dres, None, None, None, None, None,
                None, None, None, None)


def batchnorm_act(y: Tensor, st: BNStats, bn, relu: bool, residual: Optional[Tensor] = None,
                  y2: Optional[Tensor] = None, st2: Optional[BNStats] = None, bn2=None,
                  token: Optional[BNActToken] = None,
                  res_give: Optional[ResidualSlot] = None, lazy: bool = False) -> Tensor:
    """z = relu?( bn(y) [+ residual | + bn2(y2)] ).  ``token``: z's single consumer will fuse
    this BN's backward reductions; ``res_give``: slot receiving the residual's gradient.
    ``lazy``: the apply is folded into z's single consuming 1x1 conv — the returned tensor is an
    alias of y (see nn.conv_bn_act(fold_next=))."""
    return _BNActFn.apply(y, bn.weight, bn.bias, residual, y2,
                          None if bn2 is None else bn2.weight,
                          None if bn2 is None else bn2.bias, st, st2, relu, bn, token, res_give,
                          lazy)


def channel_partials(y: Tensor, shift: Tensor) -> Tuple[Tensor, Tensor]:
    """Shifted per-channel sums of an NHWC tensor (BN without a producing conv)."""
    C = y.shape[-1]
    d = y.detach().reshape(-1, C).float() - shift.float()
    return d.sum(0, keepdim=True), (d * d).sum(0, keepdim=True)


class _BNGenericFn(Function):
    """BatchNorm (+ReLU / ReLU6) over NHWC activations with any channel count (vision.hip):
    statistics kernel -> bn_finalize (running stats, num_batches_tracked) -> one affine +
    activation pass; backward = one reduction pass + one apply pass."""

    @staticmethod
    def forward(ctx, y, gamma, beta, bn, act):
        C = y.shape[-1]
        count = y.numel() // C
        if bn.training:
            ps, pss = K.chan_stats(y, bn.running_mean)
            st = bn_stats_from_partials(ps, pss, count, bn, True)
        else:
            st = bn_stats_from_partials(None, None, count, bn, False)
        z = K.affine_act(y, st.scale, st.bias, act)
        ctx.save_for_backward(y, z if act != "none" else None, gamma)
        ctx.st, ctx.act = st, act
        return z

    @staticmethod
    def backward(ctx, dz):
        y, z, gamma = ctx.saved_tensors
        st, act = ctx.st, ctx.act
        dz = dz.contiguous()
        sg, sgx = K.bn_generic_bwd_reduce(dz, z, y, st.mean, st.invstd, act)
        gd = gamma.detach()
        if st.batch_stats:
            dy = K.bn_generic_bwd_apply(dz, z, y, st.mean, st.invstd, gd, sg, sgx, st.count, act)
        else:
            dy = K.bn_generic_bwd_apply(dz, z, y, st.mean, st.invstd, gd, None, None, st.count,
                                        act)
        return dy, sgx.to(gamma.dtype), sg.to(gamma.dtype), None, None


def bn_act(y: Tensor, bn, act: str = "none") -> Tensor:
    """act(BatchNorm(y)) for NHWC ``y`` with any channel count (torch BatchNorm2d semantics:
    batch statistics + running-stat update in training, running statistics in eval)."""
    if bn.running_mean is None:
        raise NotImplementedError("BatchNorm without running statistics")
    return _BNGenericFn.apply(y, bn.weight, bn.bias, bn, act)


# ----------------------------------------------------------------------------- pooling
class _MaxPoolFn(Function):
    @staticmethod
    def forward(ctx, x, k, stride, pad, ceil_mode=False):
        y, idx = K.maxpool_fwd(x, k, stride, pad, ceil_mode)
        ctx.save_for_backward(idx)
        ctx.xshape = tuple(x.shape)
        ctx.conf = (k, stride, pad)
        ctx.mark_non_differentiable(idx)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        return K.maxpool_bwd(dy.contiguous(), idx, ctx.xshape, *ctx.conf), None, None, None, None


class _PoolBNFn(Function):
    """maxpool_k,s,p(relu(bn(y))) in one pass (the ResNet stem: BN1 + ReLU + 3x3/2 max-pool);
    the backward gathers over the pooling windows twice (Σg / Σg·x̂, then dy) instead of
    scattering dz, reducing and applying over the full-resolution tensors (pool.hip)."""

    @staticmethod
    def forward(ctx, y, gamma, beta, st, bn, k, stride, pad):
        out, idx = K.pool_bn_fwd(y, st.scale, st.bias, k, stride, pad)
        ctx.save_for_backward(y, out, idx, gamma)
        ctx.st, ctx.bn, ctx.beta, ctx.conf = st, bn, beta, (k, stride, pad)
        ctx.mark_non_differentiable(idx)
        return out, idx

    @staticmethod
    def backward(ctx, dp, _didx):
        y, out, idx, gamma = ctx.saved_tensors
        st, bn = ctx.st, ctx.bn
        if not st.batch_stats:
            raise RuntimeError("pool_bn backward needs batch statistics (training mode)")
        rep = bn_workspace(bn, "bwd", dp.device)
        direct = None
        if ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            tg, tb = _direct_grad_target(gamma), _direct_grad_target(ctx.beta)
            if tg is not None and tb is not None:
                direct = (tg[1], tb[1])
        dy, sg, sgx = K.pool_bn_bwd(dp.contiguous(), idx, out, y, st.mean, st.invstd,
                                    gamma.detach().float(), rep, st.count, *ctx.conf, acc=direct)
        _ws_done(bn, "bwd")
        if direct is not None:
            fs = _direct_grad_target(gamma)[0]
            fs.grad_ready(gamma)
            fs.grad_ready(ctx.beta)
            return dy, None, None, None, None, None, None, None
        return (dy, sgx.to(gamma.dtype) if ctx.needs_input_grad[1] else None,
                sg.to(gamma.dtype) if ctx.needs_input_grad[2] else None,
                None, None, None, None, None)


def bn_relu_maxpool(y: Tensor, st: BNStats, bn, k: int, stride: int, pad: int) -> Tensor:
    """maxpool(relu(bn(y))) on NHWC ``y``: fused kernels on the GPU (training with batch
    statistics or eval), the unfused BN-apply + max-pool otherwise."""
    if (K.pool_bn_supported(y) and (st.batch_stats or not torch.is_grad_enabled())
            and st.scale.dtype == torch.float32):
        out, _ = _PoolBNFn.apply(y, bn.weight, bn.bias, st, bn, k, stride, pad)
        return out
    return max_pool2d(batchnorm_act(y, st, bn, relu=True), k, stride, pad)


_STEM_FUSED = os.environ.get("MIPIPE_STEM_FUSED", "1") != "0"


def set_stem_fused(on: bool) -> None:
    """Route the packed ResNet stem to the recompute-fused kernels (default on)."""
    global _STEM_FUSED
    _STEM_FUSED = bool(on)


def stem_fused_ok(xp: Tensor, w_c: Tensor, bn) -> bool:
    """The recompute-fused stem applies: bf16 packed input that needs no gradient, the 224 px
    geometry (112 output columns), a BatchNorm with affine parameters and running statistics."""
    return (_STEM_FUSED and K.use_native(xp) and xp.dtype == torch.bfloat16
            and not xp.requires_grad and bn.affine and bn.running_mean is not None
            and bn.weight.dtype == torch.float32 and K.stem_fused_supported(xp, w_c))


class _StemFusedFn(Function):
    """maxpool_3x3/2/1(relu(bn(conv7x7/2(x)))) for the packed stem (stem.hip).  Forward: a
    statistics pass that recomputes the conv instead of storing y, then one pass that computes
    the conv again and writes y, the pooled output and argmax (BN-apply + ReLU + pool in
    registers / LDS).  Backward: the BN reduction over the POOLED gradient and output (x̂ of the
    window's argmax pixel recovered as (z-β)/γ: no pass over the 4x larger conv output), then ONE
    pass that routes the pooled gradient, forms dy = A·g + B·y + C in LDS and accumulates the
    weight gradient from it — dy never reaches HBM.  Numerics follow the unfused conv -> pool_bn
    path to bf16 rounding (x̂ from the stored bf16 z instead of the stored bf16 y)."""

    @staticmethod
    def forward(ctx, xp, weight, w_c, gamma, beta, bn):
        ws = bn_workspace(bn, "fwd", xp.device)
        ps, pss = K.stem_fwd_stats(xp, w_c, bn.running_mean, ws[0], ws[1])
        count = xp.shape[0] * ((xp.shape[1] - 7) // 2 + 1) * (xp.shape[2] - 3)
        st = bn_stats_from_partials(ps, pss, count, bn, True)
        out, idx, y = K.stem_fwd_pool(xp, w_c, st.scale, st.bias)
        ctx.save_for_backward(xp, y, out, idx, gamma)
        ctx.st, ctx.bn, ctx.weight, ctx.beta = st, bn, weight, beta
        return out

    @staticmethod
    def backward(ctx, dp):
        xp, y, out, idx, gamma = ctx.saved_tensors
        st, bn = ctx.st, ctx.bn
        rep = bn_workspace(bn, "bwd", dp.device)
        direct = None
        if ctx.needs_input_grad[3] and ctx.needs_input_grad[4]:
            tg, tb = _direct_grad_target(gamma), _direct_grad_target(ctx.beta)
            if tg is not None and tb is not None:
                direct = (tg[1], tb[1])
        dwp, sg, sgx = K.stem_bwd(xp, y, dp.contiguous(), idx, out, st.mean, st.invstd,
                                  gamma.detach(), ctx.beta.detach(), rep, st.count, acc=direct)
        _ws_done(bn, "bwd")
        dw = None
        if ctx.needs_input_grad[1]:
            dw = _wgrad_map_into_grad(ctx.weight._mipipe_wgrad_map, dwp, ctx.weight)
        if direct is not None:
            fs = _direct_grad_target(gamma)[0]
            fs.grad_ready(gamma)
            fs.grad_ready(ctx.beta)
            return None, dw, None, None, None, None
        return (None, dw, None, sgx.to(gamma.dtype) if ctx.needs_input_grad[3] else None,
                sg.to(gamma.dtype) if ctx.needs_input_grad[4] else None, None)


def stem_conv_bn_relu_maxpool(xp: Tensor, weight: Tensor, w_c: Tensor, bn) -> Tensor:
    """Fused stem on packed input ``xp`` (see :func:`stem_fused_ok`).  Training: batch statistics
    (recompute-fused forward and backward); eval: running statistics, one BN + ReLU + pool pass."""
    if bn.training:
        return _StemFusedFn.apply(xp, weight, w_c, bn.weight, bn.bias, bn)
    st = bn_stats_from_partials(None, None, 0, bn, False)
    return K.stem_fwd_pool(xp, w_c, st.scale, st.bias, want_y=False)[0]


def max_pool2d(x: Tensor, k: int, stride: int, pad: int, ceil_mode: bool = False) -> Tensor:
    return _MaxPoolFn.apply(x, k, stride, pad, bool(ceil_mode))


class _AvgPool2dFn(Function):
    @staticmethod
    def forward(ctx, x, k, stride, pad):
        ctx.conf = (tuple(x.shape), k, stride, pad)
        return K.avgpool2d_fwd(x, k, stride, pad)

    @staticmethod
    def backward(ctx, dy):
        xs, k, s, p = ctx.conf
        return K.avgpool2d_bwd(dy.contiguous(), xs, k, s, p), None, None, None


def avg_pool2d(x: Tensor, k: int, stride: Optional[int] = None, pad: int = 0) -> Tensor:
    """NHWC k x k average pool (count_include_pad=True, floor mode: torch's defaults)."""
    return _AvgPool2dFn.apply(x, int(k), int(stride or k), int(pad))


class _AvgPoolFn(Function):
    @staticmethod
    def forward(ctx, x):
        ctx.xshape = tuple(x.shape)
        return K.avgpool_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return K.avgpool_bwd(dy.contiguous(), ctx.xshape)


def global_avg_pool(x: Tensor) -> Tensor:
    """NHWC [N,H,W,C] -> [N,C] (AdaptiveAvgPool2d((1,1)) + flatten)."""
    return _AvgPoolFn.apply(x)


# ----------------------------------------------------------------------------- linear
class _LinearFn(Function):
    @staticmethod
    def forward(ctx, x, weight, w_c, bias, act, bias_c, res_take, bias_slot):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        bk = bias if bias_c is None else bias_c  # bias_c: the kernel's (padded) bias vector
        pf = _prefetch.before_weight_gemm(w_c)  # the next GEMM's weight, warmed by this one
        if act == "gelu":  # GELU in the GEMM epilogue (h, the pre-activation, saved)
            y, h = K.gemm_gelu(x2.contiguous(), w_c, bk, prefetch=pf)
            ctx.save_for_backward(x2, w_c, h)
        else:
            y = K.gemm(x2, w_c, False, True, bk, act, x.dtype, prefetch=pf)
            ctx.save_for_backward(x2, w_c, y if act == "relu" else None)
        ctx.act, ctx.shp, ctx.has_bias = act, shp, bias is not None
        ctx.weight, ctx.bias = weight, bias
        ctx.res_take = res_take
        ctx.bias_slot = bias_slot
        if bias_slot is not None:  # the consuming LayerNorm may sum this bias's gradient
            bias_slot.bias = bias if bias_c is None and act == "none" else None
            bias_slot.done = False
        return y.reshape(*shp[:-1], y.shape[-1])

    @staticmethod
    def backward(ctx, dy):
        x2, w_c, aux = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1]).contiguous()
        # the bias gradient's flat-space target (native path): a GELU layer sums it in the GELU
        # backward's own pass over dy instead of a separate colsum over the result
        tb = None
        if ctx.has_bias and ctx.needs_input_grad[3] and K.use_native(dy2):
            tb = _direct_grad_target(ctx.bias, dy2.shape[1])
        bias_done = ctx.bias_slot is not None and ctx.bias_slot.done
        if ctx.act == "gelu":
            if tb is not None and K.gelu_bwd_colsum_ok(dy2):
                dy2 = K.gelu_bwd_colsum(dy2, aux, tb[1])
                bias_done = True
            else:
                dy2 = K.gelu_bwd(dy2, aux)
        elif ctx.act == "relu":
            dy2 = (dy2.float() * (aux > 0)).to(dy2.dtype)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # the input's other gradient (residual stream), handed over by the consumer that ran
            # first, is added in the data-grad GEMM's epilogue
            add = ctx.res_take.take() if ctx.res_take is not None else None
            if add is not None:
                add = add.reshape(-1, add.shape[-1]).to(dy2.dtype).contiguous()
            # (the weight-grad GEMM below reads the saved input next: warmed by this one)
            pf = _prefetch.before_weight_gemm(w_c, [x2] if ctx.needs_input_grad[1] else None)
            dx = K.gemm(dy2, w_c, False, False, None, "none", dy2.dtype,
                        addend=add, prefetch=pf).reshape(ctx.shp)
        gdt = torch.float64 if dy2.dtype == torch.float64 else torch.float32
        if ctx.needs_input_grad[1]:
            # w_c may carry more rows than the parameter (vocabulary padded to the tile width):
            # then the target is the flat space's padded gradient view
            tgt = _direct_grad_target(ctx.weight, w_c.shape[0]) if K.use_native(dy2) else None
            # a tied weight (``_mipipe_tied_later``: an MLM decoder sharing the input embedding)
            # gets another contribution later in the backward — that writer reports it ready,
            # else DDP would all-reduce a partial gradient.  Unless DDP takes the lookup part as
            # sparse rows (``_mipipe_sparse_sink``): then this dense part is the whole local
            # gradient of the weight and it is ready now (its bucket overlaps the encoder's
            # backward instead of being all-reduced after the last kernel).
            sink = getattr(ctx.weight, "_mipipe_sparse_sink", None)
            ready_now = sink is not None or not getattr(ctx.weight, "_mipipe_tied_later", False)
            if tgt is not None:
                fs, g = tgt
                K.gemm(dy2, x2, True, False, None, "none", torch.float32,
                       g.reshape(w_c.shape[0], -1), 1.0)
                if ready_now:
                    fs.grad_ready(ctx.weight)
            else:
                dw = K.gemm(dy2, x2, True, False, None, "none", gdt)
                if w_c.shape[0] != ctx.weight.shape[0]:
                    dw = dw[: ctx.weight.shape[0]]
                if sink is not None:  # write it into the flat gradient now, report it ready
                    from mipipe.optim.flat import flat_space_for
                    fs = flat_space_for(ctx.weight)
                    fs.grad_view(ctx.weight).add_(dw.to(torch.float32))
                    fs.grad_ready(ctx.weight)
                    dw = None
        if ctx.has_bias and ctx.needs_input_grad[3]:
            if tb is not None:
                if not bias_done:
                    K.colsum(dy2, tb[1])
                tb[0].grad_ready(ctx.bias)
            else:
                db = K.colsum(dy2)
                if ctx.bias.shape[0] != db.shape[0]:
                    db = db[: ctx.bias.shape[0]]
                db = db.to(gdt)
        return dx, dw, None, db, None, None, None, None


def linear(x: Tensor, weight: Tensor, w_c: Tensor, bias: Optional[Tensor], act: str = "none",
           bias_c: Optional[Tensor] = None, res_take: Optional["ResidualSlot"] = None,
           bias_slot: Optional[BiasGradSlot] = None):
    """y = act(x @ w_c^T + bias).  ``weight`` / ``bias``: the parameters (gradient targets);
    ``w_c``: the compute-dtype operand, ``bias_c``: the bias vector the kernel reads (both may
    be padded along the output dimension — a vocabulary rounded up to the tile width).
    ``res_take``: x is also consumed elsewhere (a residual stream); that consumer's gradient
    wrt x, handed over through the slot, is added in this layer's data-grad GEMM.
    ``bias_slot``: the output feeds :func:`layer_norm` with the same slot, whose backward
    computes this layer's bias gradient."""
    return _LinearFn.apply(x, weight, w_c, bias, act, bias_c, res_take, bias_slot)


# ----------------------------------------------------------------------------- loss
class _CrossEntropyFn(Function):
    """Native: the forward keeps the logits and per-row log-sum-exps, the backward writes the
    scaled gradient in one pass (upstream gradient read on the device; no [R, V] gradient from
    the forward and no separate rescale).  Fallback: fused fwd+bwd reference, rescaled."""

    @staticmethod
    def forward(ctx, logits, labels, label_smoothing, ignore_index, valid_cols):
        logits, labels = logits.contiguous(), labels.contiguous()
        ctx.args = (label_smoothing, ignore_index, valid_cols)
        ctx.split = K.use_native(logits)
        if ctx.split:
            loss, work = K.native().cross_entropy_fwd(logits, labels, label_smoothing,
                                                      ignore_index, valid_cols)
            ctx.save_for_backward(logits, labels, work)
            return loss
        loss, grad = K.cross_entropy_fwd_bwd(logits, labels, label_smoothing, ignore_index,
                                             valid_cols)
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        if ctx.split:
            logits, labels, work = ctx.saved_tensors
            gout = g.detach().reshape(1).to(torch.float32)
            return (K.native().cross_entropy_bwd(logits, labels, work, gout, *ctx.args),
                    None, None, None, None)
        (grad,) = ctx.saved_tensors
        return (grad * g.to(grad.dtype)), None, None, None, None


def cross_entropy(logits: Tensor, labels: Tensor, label_smoothing: float = 0.0,
                  ignore_index: int = -100, valid_cols: int = -1) -> Tensor:
    """Fused log-softmax + NLL (mean) whose backward costs one scale.  ``valid_cols``: classes
    are the first columns only (tile-padded vocabulary)."""
    return _CrossEntropyFn.apply(logits, labels, label_smoothing, ignore_index, int(valid_cols))


# ----------------------------------------------------------------------------- transformer ops
class _LayerNormFn(Function):
    @staticmethod
    def forward(ctx, x, gamma, beta, eps, residual, res_give, drop, bias_slot):
        y, mean, rstd, xs = K.layernorm_fwd(x, gamma, beta, eps, residual, drop)
        ctx.save_for_backward(x if xs is None else xs, mean, rstd, gamma)
        ctx.beta = beta
        ctx.has_res = residual is not None
        ctx.res_give = res_give
        ctx.drop = drop
        ctx.bias_slot = bias_slot
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, rstd, gamma = ctx.saved_tensors
        acc = None
        if K.use_native(dy) and ctx.needs_input_grad[1] and ctx.needs_input_grad[2]:
            tg, tb = _direct_grad_target(gamma), _direct_grad_target(ctx.beta)
            if tg is not None and tb is not None:
                acc = (tg[1], tb[1])
        # the producing Linear's bias gradient, summed in this kernel (native, flat space only)
        slot, tbias = ctx.bias_slot, None
        if acc is not None and slot is not None and slot.bias is not None:
            tbias = _direct_grad_target(slot.bias, x.shape[-1])
        dx, dgamma, dbeta, dxd = K.layernorm_bwd(dy.contiguous(), x, mean, rstd, gamma, acc,
                                                 ctx.drop, None if tbias is None else tbias[1])
        if tbias is not None:
            slot.done = True
        dres = None
        if ctx.has_res:
            # d/d residual = d/dx; handed to the residual's other consumer when it fuses the add
            dres = ctx.res_give.produce(dx) if ctx.res_give is not None else dx
        dxin = dxd if dxd is not None else dx  # fused dropout: the dropped branch's gradient
        if acc is not None:
            fs = _direct_grad_target(gamma)[0]
            fs.grad_ready(gamma)
            fs.grad_ready(ctx.beta)
            return dxin, None, None, None, dres, None, None, None
        return dxin, dgamma.to(gamma.dtype), dbeta.to(gamma.dtype), None, dres, None, None, None


def layer_norm(x: Tensor, gamma: Tensor, beta: Tensor, eps: float = 1e-12,
               residual: Optional[Tensor] = None,
               res_give: Optional["ResidualSlot"] = None, dropout_p: float = 0.0,
               dropout_seed=None, bias_slot: Optional[BiasGradSlot] = None) -> Tensor:
    """LN(dropout(x) [+ residual]) — BERT's post-LN residual branch (dropout, add, norm) in one
    kernel each way.  ``res_give``: the residual's gradient goes to the slot (for the residual's
    other consumer to add in its own kernel) instead of through autograd.  ``dropout_p`` > 0
    (with ``residual``): the branch's dropout, mask identical to :func:`dropout` with that
    seed.  ``bias_slot``: x is the output of :func:`linear` given the same slot; this backward
    also computes that layer's bias gradient."""
    drop = None
    if dropout_p > 0.0:
        if residual is None:
            x = dropout(x, dropout_p, dropout_seed)
            bias_slot = None  # the branch gradient is not this kernel's any more
        else:
            seed = dropout_seed if isinstance(dropout_seed, K.DevSeed) \
                else int(dropout_seed) & 0xFFFFFFFF
            drop = (float(dropout_p), seed)
    return _LayerNormFn.apply(x, gamma, beta, eps, residual, res_give, drop, bias_slot)


class _GeluFn(Function):
    @staticmethod
    def forward(ctx, x):
        ctx.save_for_backward(x)
        return K.gelu_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        return K.gelu_bwd(dy.contiguous(), x)


def gelu(x: Tensor) -> Tensor:
    return _GeluFn.apply(x)


class _AttentionFn(Function):
    @staticmethod
    def forward(ctx, qkv, B, S, H, mask, scale, p_drop, seed):
        o, lse = K.attention_fwd(qkv, B, S, H, mask, scale, p_drop, seed)
        ctx.save_for_backward(qkv, o, lse, mask)
        ctx.cfg = (B, S, H, scale, p_drop, seed)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, o, lse, mask = ctx.saved_tensors
        B, S, H, scale, p_drop, seed = ctx.cfg
        dqkv = K.attention_bwd(do.contiguous(), qkv, o, lse, B, S, H, mask, scale, p_drop, seed)
        return dqkv, None, None, None, None, None, None, None


def attention(qkv: Tensor, batch: int, seq: int, heads: int, mask: Optional[Tensor] = None,
              scale: Optional[float] = None, p_drop: float = 0.0, seed: int = 0) -> Tensor:
    """Fused softmax(QKᵀ·scale + mask)·V over the packed QKV projection output.

    qkv [B*S, 3*H*D] (q | k | v column blocks, head-major), mask [B, S] additive key bias
    (0 / -inf style) -> o [B*S, H*D], ready for the output projection.  ``p_drop`` is the
    attention-probability dropout (keyed by ``seed``; recomputed in the backward)."""
    D = qkv.shape[-1] // (3 * heads)
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    if mask is not None:
        mask = mask.float().contiguous()
    if not isinstance(seed, K.DevSeed):
        seed = int(seed) & 0xFFFFFFFF
    return _AttentionFn.apply(qkv.contiguous(), batch, seq, heads, mask, float(scale),
                              float(p_drop), seed)


class _DropoutFn(Function):
    @staticmethod
    def forward(ctx, x, p, seed):
        ctx.cfg = (p, seed)
        return K.dropout_fwd(x.contiguous(), p, seed)

    @staticmethod
    def backward(ctx, dy):
        p, seed = ctx.cfg
        return K.dropout_fwd(dy.contiguous(), p, seed), None, None


def dropout(x: Tensor, p: float, seed: int, training: bool = True) -> Tensor:
    """Hash-keyed dropout: the mask is a pure function of (seed, element index), so the backward
    regenerates it instead of storing it."""
    if not training or p <= 0.0:
        return x
    if not isinstance(seed, K.DevSeed):
        seed = int(seed) & 0xFFFFFFFF
    return _DropoutFn.apply(x, float(p), seed)


class _EmbeddingFn(Function):
    @staticmethod
    def forward(ctx, idx, weight, w_c):
        ctx.save_for_backward(idx)
        ctx.rows = weight.shape[0]
        ctx.weight = weight
        return w_c[idx]

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        sink = getattr(ctx.weight, "_mipipe_sparse_sink", None)
        if ctx.needs_input_grad[1] and sink is not None:
            # DDP exchanges the lookup gradient as (token id, row) pairs and scatters every
            # rank's rows after the dense part's all-reduce (parallel/ddp.py)
            sink(idx, dy)
            return None, None, None
        if ctx.needs_input_grad[1] and K.use_native(dy):
            tgt = _direct_grad_target(ctx.weight)
            if tgt is not None:  # scatter straight into the flat gradient buffer
                K.embedding_bwd(dy.contiguous(), idx, ctx.rows, tgt[1])
                tgt[0].grad_ready(ctx.weight)
                return None, None, None
        return None, K.embedding_bwd(dy.contiguous(), idx, ctx.rows), None


def embedding(idx: Tensor, weight: Tensor, w_c: Tensor) -> Tensor:
    sink = getattr(weight, "_mipipe_sparse_sink", None)
    if sink is not None and weight.requires_grad and torch.is_grad_enabled():
        sink.on_forward(idx)  # DDP: the ids' all_gather starts with the forward
    return _EmbeddingFn.apply(idx, weight, w_c)
