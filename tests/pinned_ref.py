"""Decision-pinned float64 reference for ResNet-18/34 training steps.

A fp32 GPU forward and a float64 forward of the same weights differ by ~1e-7 relative, so a
ReLU whose pre-activation lies within that distance of 0 (or a max-pool window whose two best
values do) may decide differently in the two evaluations.  One flipped decision routes a full
gradient element differently and moves a small tensor's gradient by ~1/count (1e-2 for a layer4
BatchNorm at batch 64) — a legitimate difference that says nothing about the kernels' arithmetic.

This module evaluates the reference (task.py:309-311: conv -> BN -> ReLU blocks, 3x3/2 max-pool
stem, avgpool, fc, cross-entropy) in float64 with plain torch ops and autograd, but takes every
DECISION from the GPU run: the ReLU masks (z > 0 of each fused BN+ReLU output) and the stem
max-pool's window argmax.  Any remaining gradient difference is arithmetic.

``record_gpu_decisions`` wraps the two kernel entry points that take decisions on the fp32 GPU
path (``kernels.bn_act_fwd`` — every BN(+residual)+ReLU of the blocks — and
``kernels.pool_bn_fwd`` — the stem's BN+ReLU+max-pool) and returns the tape in call order.
"""
from __future__ import annotations

import contextlib
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F


class DecisionTape:
    def __init__(self):
        self.relu_masks: List[torch.Tensor] = []   # NCHW bool, block order (conv1, conv2) x blocks
        self.pool: Optional[tuple] = None          # (tap index NCHW int64, out > 0 NCHW bool)

    def summary(self) -> str:
        n = sum(int(m.numel()) for m in self.relu_masks)
        return f"{len(self.relu_masks)} relu masks ({n} decisions), pool={'yes' if self.pool else 'no'}"


@contextlib.contextmanager
def record_gpu_decisions():
    from mipipe.ops import kernels as K
    tape = DecisionTape()
    orig_act, orig_pool = K.bn_act_fwd, K.pool_bn_fwd

    def bn_act_fwd(y, scale, bias, relu, *a, **kw):
        z = orig_act(y, scale, bias, relu, *a, **kw)
        if relu:
            tape.relu_masks.append((z > 0).permute(0, 3, 1, 2).cpu())
        return z

    def pool_bn_fwd(y, scale, bias, k, stride, pad):
        out, idx = orig_pool(y, scale, bias, k, stride, pad)
        assert tape.pool is None, "one stem pool per forward"
        tape.pool = (idx.permute(0, 3, 1, 2).long().cpu(), (out > 0).permute(0, 3, 1, 2).cpu(),
                     (k, stride, pad))
        return out, idx

    K.bn_act_fwd, K.pool_bn_fwd = bn_act_fwd, pool_bn_fwd
    try:
        yield tape
    finally:
        K.bn_act_fwd, K.pool_bn_fwd = orig_act, orig_pool


def _bn_train(y, w, b, eps=1e-5):
    mean = y.mean((0, 2, 3), keepdim=True)
    var = y.var((0, 2, 3), unbiased=False, keepdim=True)
    return (y - mean) * torch.rsqrt(var + eps) * w.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)


class _Pinner:
    """Applies recorded decisions in order; with ``tape=None`` it takes its own (float64)
    decisions and records them, so the pinned reference can be checked against plain autograd."""

    def __init__(self, tape: Optional[DecisionTape]):
        self.tape = tape
        self.own = DecisionTape() if tape is None else None
        self.i = 0

    def relu(self, a):
        if self.tape is None:
            m = a > 0
            self.own.relu_masks.append(m.detach())
        else:
            m = self.tape.relu_masks[self.i]
            assert m.shape == a.shape, (self.i, m.shape, a.shape)
        self.i += 1
        return torch.where(m, a, torch.zeros((), dtype=a.dtype))

    def maxpool(self, a, k, s, p):
        N, C, H, W = a.shape
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        if self.tape is None:
            z = torch.relu(a)
            zp = F.pad(z, (p, p, p, p), value=-1.0)   # relu'd values are >= 0: pads never win
            taps = torch.stack([zp[:, :, kh:kh + s * (Ho - 1) + 1:s, kw:kw + s * (Wo - 1) + 1:s]
                                for kh in range(k) for kw in range(k)], 0)
            idx = taps.argmax(0)  # first maximum, like the kernel's strict '>'
            pos = torch.gather(taps, 0, idx[None])[0] > 0
            self.own.pool = (idx.detach(), pos.detach(), (k, s, p))
        else:
            idx, pos, geo = self.tape.pool
            assert geo == (k, s, p) and idx.shape == (N, C, Ho, Wo)
        ap = F.pad(a, (p, p, p, p))
        out = torch.zeros(N, C, Ho, Wo, dtype=a.dtype)
        for kh in range(k):
            for kw in range(k):
                tap = ap[:, :, kh:kh + s * (Ho - 1) + 1:s, kw:kw + s * (Wo - 1) + 1:s]
                out = out + torch.where(idx == kh * k + kw, tap, torch.zeros((), dtype=a.dtype))
        return torch.where(pos, out, torch.zeros((), dtype=a.dtype))


def resnet_basic_forward(P: Dict[str, torch.Tensor], x: torch.Tensor, layers=(2, 2, 2, 2),
                         tape: Optional[DecisionTape] = None):
    """torchvision ResNet (BasicBlock) forward in the dtype of ``P`` (NCHW), decisions pinned to
    ``tape``.  Returns (logits, pinner)."""
    pin = _Pinner(tape)
    a = _bn_train(F.conv2d(x, P["conv1.weight"], stride=2, padding=3), P["bn1.weight"],
                  P["bn1.bias"])
    h = pin.maxpool(a, 3, 2, 1)
    for li, nb in enumerate(layers, start=1):
        for bi in range(nb):
            pre = f"layer{li}.{bi}."
            stride = 2 if (li > 1 and bi == 0) else 1
            o = F.conv2d(h, P[pre + "conv1.weight"], stride=stride, padding=1)
            o = pin.relu(_bn_train(o, P[pre + "bn1.weight"], P[pre + "bn1.bias"]))
            o = _bn_train(F.conv2d(o, P[pre + "conv2.weight"], padding=1), P[pre + "bn2.weight"],
                          P[pre + "bn2.bias"])
            if pre + "downsample.0.weight" in P:
                idn = _bn_train(F.conv2d(h, P[pre + "downsample.0.weight"], stride=stride),
                                P[pre + "downsample.1.weight"], P[pre + "downsample.1.bias"])
            else:
                idn = h
            h = pin.relu(o + idn)
    feat = h.mean((2, 3))
    return F.linear(feat, P["fc.weight"], P["fc.bias"]), pin


def pinned_grads(state: Dict[str, torch.Tensor], param_names, x, labels, tape, layers=(2, 2, 2, 2)):
    """float64 loss and parameter gradients of one training step with ``tape``'s decisions."""
    P = {k: v.detach().double().cpu().clone() for k, v in state.items()}
    for n in param_names:
        P[n].requires_grad_(True)
    logits, pin = resnet_basic_forward(P, x.double().cpu(), layers, tape)
    if tape is not None:
        assert pin.i == len(tape.relu_masks), (pin.i, len(tape.relu_masks))
    loss = F.cross_entropy(logits, labels.cpu())
    loss.backward()
    return logits.detach(), loss.detach(), {n: P[n].grad for n in param_names}, pin


def flipped_decisions(tape: DecisionTape, own: DecisionTape) -> Dict[str, int]:
    """How many decisions of ``tape`` differ from ``own`` (float64's), per site."""
    out = {}
    for i, (a, b) in enumerate(zip(tape.relu_masks, own.relu_masks)):
        n = int((a != b).sum())
        if n:
            out[f"relu[{i}]"] = n
    if tape.pool is not None and own.pool is not None:
        ia, pa, _ = tape.pool
        ib, pb, _ = own.pool
        n = int(((ia != ib) & pa).sum() + (pa != pb).sum())
        if n:
            out["stem_pool"] = n
    return out
