"""Reference (plain PyTorch) implementations of mipipe's kernel contracts.

Every hot op of the training step is a hand-written HIP kernel on the MI355X
(``csrc/kernels/*.hip`` -> ``mipipe._C``).  This module implements the *same contracts*
(same arguments, layouts, outputs) with ATen math.  It is used

* as the CPU execution path (CPU/gloo configs, tests without a GPU), and
* as the fp32 numerics oracle the GPU tests compare each kernel against.

Layout conventions shared with the kernels: activations are NHWC (``[N, H, W, C]``,
C contiguous); conv weights are ``[Cout, KH, KW, Cin]`` (the channels_last physical order of
a torch ``[Cout, Cin, KH, KW]`` parameter); BN statistics are per channel.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


def _f(t: Tensor) -> Tensor:
    """Upcast low-precision tensors to fp32; keep fp64 (used by exactness tests)."""
    return t if t.dtype == torch.float64 else t.float()


def _nchw(x: Tensor) -> Tensor:
    return x.permute(0, 3, 1, 2)


def _nhwc(x: Tensor) -> Tensor:
    return x.permute(0, 2, 3, 1).contiguous()


def _w_oihw(w: Tensor) -> Tensor:
    return w.permute(0, 3, 1, 2)


def conv_fwd(x: Tensor, w: Tensor, stride: int, pad: int,
             stats_shift: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor], Optional[Tensor]]:
    """y = conv(x, w).  Returns (y, Σ(y-shift), Σ(y-shift)²) per channel ([1, Co] fp32 partials)
    when ``stats_shift`` is given (BN-stat epilogue), else (y, None, None)."""
    yf = F.conv2d(_f(_nchw(x)), _f(_w_oihw(w)), stride=stride, padding=pad)
    y = _nhwc(yf)
    if stats_shift is None:
        return y.to(x.dtype), None, None
    d = y.reshape(-1, y.shape[-1]) - _f(stats_shift)[None, :]
    return y.to(x.dtype), d.sum(0, keepdim=True), (d * d).sum(0, keepdim=True)


def conv_dgrad(dy: Tensor, w: Tensor, x_shape, stride: int, pad: int) -> Tensor:
    N, H, W, Ci = x_shape
    dx = torch.nn.grad.conv2d_input((N, Ci, H, W), _f(_w_oihw(w)), _f(_nchw(dy)),
                                    stride=stride, padding=pad)
    return _nhwc(dx).to(dy.dtype)


def conv_wgrad(dy: Tensor, x: Tensor, kh: int, kw: int, stride: int, pad: int) -> Tensor:
    Co = dy.shape[-1]
    Ci = x.shape[-1]
    dw = torch.nn.grad.conv2d_weight(_f(_nchw(x)), (Co, Ci, kh, kw), _f(_nchw(dy)),
                                     stride=stride, padding=pad)
    return dw.permute(0, 2, 3, 1).contiguous()  # [Co, KH, KW, Ci] fp32


def bn_finalize(psum: Tensor, psumsq: Tensor, count: int, shift: Tensor, gamma: Tensor,
                beta: Tensor, running_mean: Optional[Tensor], running_var: Optional[Tensor],
                momentum: float, eps: float) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Batch statistics from shifted partial sums; updates running stats in place
    (unbiased variance, torch semantics).  Returns (mean, invstd, scale, bias) with
    ``bn(y) = y*scale + bias``."""
    s = _f(psum).sum(0)
    ss = _f(psumsq).sum(0)
    m_shift = s / count
    var = (ss / count - m_shift * m_shift).clamp_min(0.0)
    mean = m_shift + _f(shift)
    invstd = torch.rsqrt(var + eps)
    scale = _f(gamma) * invstd
    bias = _f(beta) - mean * scale
    if running_mean is not None:
        with torch.no_grad():
            unbiased = var * (count / max(count - 1, 1))
            running_mean.mul_(1 - momentum).add_(mean.to(running_mean.dtype), alpha=momentum)
            running_var.mul_(1 - momentum).add_(unbiased.to(running_var.dtype), alpha=momentum)
    return mean, invstd, scale, bias


def bn_act_fwd(y: Tensor, scale: Tensor, bias: Tensor, relu: bool,
               residual: Optional[Tensor] = None, res_scale: Optional[Tensor] = None,
               res_bias: Optional[Tensor] = None) -> Tensor:
    """z = act(y*scale + bias [+ residual | + residual*res_scale + res_bias])."""
    z = _f(y) * scale + bias
    if residual is not None:
        r = _f(residual)
        if res_scale is not None:
            r = r * res_scale + res_bias
        z = z + r
    if relu:
        z = torch.relu(z)
    return z.to(y.dtype)


def bn_act_bwd_reduce(dz: Tensor, z: Tensor, y: Tensor, mean: Tensor, invstd: Tensor,
                      relu: bool) -> Tuple[Tensor, Tensor]:
    """Σ g and Σ g·x̂ per channel, g = dz·[z>0] (relu) or dz, x̂ = (y-mean)·invstd."""
    C = y.shape[-1]
    g = _f(dz).reshape(-1, C)
    if relu:
        g = g * (z.reshape(-1, C) > 0)
    xhat = (_f(y).reshape(-1, C) - mean) * invstd
    return g.sum(0), (g * xhat).sum(0)


def bn_act_bwd_apply(dz: Tensor, z: Tensor, y: Tensor, mean: Tensor, invstd: Tensor,
                     gamma: Tensor, sum_g: Tensor, sum_gx: Tensor, count: int, relu: bool,
                     want_dres: bool = False) -> Tuple[Tensor, Optional[Tensor]]:
    """dy = γ·invstd·(g − Σg/n − x̂·Σgx̂/n); optionally d(residual) = g."""
    shp = y.shape
    C = shp[-1]
    g = _f(dz).reshape(-1, C)
    if relu:
        g = g * (z.reshape(-1, C) > 0)
    xhat = (_f(y).reshape(-1, C) - mean) * invstd
    dy = (_f(gamma) * invstd) * (g - sum_g / count - xhat * (sum_gx / count))
    dres = g.reshape(shp).to(dz.dtype) if want_dres else None
    return dy.reshape(shp).to(dz.dtype), dres


def relu_mask_grad(dz: Tensor, z: Tensor) -> Tensor:
    return (_f(dz) * (z > 0)).to(dz.dtype)


def maxpool_fwd(x: Tensor, k: int, stride: int, pad: int,
                ceil_mode: bool = False) -> Tuple[Tensor, Tensor]:
    yf, idx = F.max_pool2d(_f(_nchw(x)), k, stride, pad, ceil_mode=ceil_mode,
                           return_indices=True)
    return _nhwc(yf).to(x.dtype), _nhwc(idx.to(torch.int32))


def maxpool_bwd(dy: Tensor, idx: Tensor, x_shape) -> Tensor:
    N, H, W, C = x_shape
    dyf = _f(_nchw(dy)).reshape(N, C, -1)
    dx = torch.zeros(N, C, H * W, dtype=dyf.dtype, device=dy.device)
    dx.scatter_add_(2, _nchw(idx).reshape(N, C, -1).long(), dyf)
    return _nhwc(dx.reshape(N, C, H, W)).to(dy.dtype)


def avgpool_fwd(x: Tensor) -> Tensor:
    """Global average pool NHWC -> [N, C]."""
    return _f(x).mean(dim=(1, 2)).to(x.dtype)


def avgpool_bwd(dy: Tensor, x_shape) -> Tensor:
    N, H, W, C = x_shape
    return (_f(dy)[:, None, None, :] / (H * W)).expand(N, H, W, C).contiguous().to(dy.dtype)


def gemm(a: Tensor, b: Tensor, trans_a: bool, trans_b: bool, bias: Optional[Tensor] = None,
         act: str = "none", out_dtype=None, c: Optional[Tensor] = None,
         beta: float = 0.0) -> Tensor:
    """C = op(A)·op(B) (+bias per column) (+act) (+beta·C).  A: [M,K] or [K,M]."""
    A = _f(a).t() if trans_a else _f(a)
    B = _f(b).t() if trans_b else _f(b)
    out = A @ B
    if bias is not None:
        out = out + _f(bias)
    if act == "relu":
        out = torch.relu(out)
    elif act == "gelu":
        out = F.gelu(out)
    if c is not None and beta != 0.0:
        out = out + beta * _f(c)
    return out.to(out_dtype or a.dtype)


def cross_entropy_fwd_bwd(logits: Tensor, labels: Tensor, label_smoothing: float = 0.0,
                          ignore_index: int = -100,
                          valid_cols: int = -1) -> Tuple[Tensor, Tensor]:
    """Mean CE over non-ignored rows and its gradient wrt logits (for grad_output = 1).
    ``valid_cols`` > 0: only the first columns are classes; the gradient of the rest is 0."""
    V = logits.shape[-1]
    if 0 < valid_cols < V:
        loss, g = cross_entropy_fwd_bwd(logits[:, :valid_cols], labels, label_smoothing,
                                        ignore_index)
        return loss, torch.cat([g, g.new_zeros(g.shape[0], V - valid_cols)], 1)
    lf = _f(logits)
    valid = labels != ignore_index
    n = valid.sum().clamp_min(1)
    logp = torch.log_softmax(lf, dim=-1)
    safe = labels.clamp_min(0).long()
    nll = -logp.gather(1, safe[:, None])[:, 0]
    if label_smoothing > 0:
        smooth = -logp.mean(dim=-1)
        nll = (1 - label_smoothing) * nll + label_smoothing * smooth
    loss = (nll * valid).sum() / n
    p = logp.exp()
    oh = F.one_hot(safe, lf.shape[-1]).float()
    if label_smoothing > 0:
        oh = oh * (1 - label_smoothing) + label_smoothing / lf.shape[-1]
    grad = (p - oh) * valid[:, None] / n
    return loss, grad.to(logits.dtype)


def sgd_step(param: Tensor, grad: Tensor, mom: Tensor, shadow: Optional[Tensor], lr: float,
             momentum: float, dampening: float, weight_decay: float, nesterov: bool,
             first_step: bool, grad_scale: float = 1.0) -> None:
    """torch.optim.SGD semantics ([torch] optim/sgd.py:354-380) on flat buffers; also refreshes
    the bf16 compute shadow of the parameters."""
    g = _f(grad) * grad_scale
    if weight_decay != 0:
        g = g + weight_decay * param
    if momentum != 0:
        if first_step:
            mom.copy_(g)
        else:
            mom.mul_(momentum).add_(g, alpha=1 - dampening)
        g = g + momentum * mom if nesterov else mom
    param.add_(g, alpha=-lr)
    if shadow is not None:
        shadow.copy_(param.to(shadow.dtype))


def adamw_step(param: Tensor, grad: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor,
               shadow: Optional[Tensor], lr: float, beta1: float, beta2: float, eps: float,
               weight_decay: float, step: int, grad_scale: float = 1.0) -> None:
    g = _f(grad) * grad_scale
    param.mul_(1 - lr * weight_decay)
    exp_avg.mul_(beta1).add_(g, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    param.addcdiv_(exp_avg, denom, value=-lr / bc1)
    if shadow is not None:
        shadow.copy_(param.to(shadow.dtype))


def layernorm_fwd(x: Tensor, gamma: Tensor, beta: Tensor, eps: float,
                  residual: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor, Optional[Tensor]]:
    """(y, mean, rstd, x_sum): y = LN(x [+ residual]); x_sum = x+residual (saved for bwd)."""
    xs = _f(x) if residual is None else _f(x) + _f(residual)
    mean = xs.mean(-1)
    var = xs.var(-1, unbiased=False)
    rstd = torch.rsqrt(var + eps)
    y = (xs - mean[..., None]) * rstd[..., None] * _f(gamma) + _f(beta)
    return y.to(x.dtype), mean, rstd, (xs.to(x.dtype) if residual is not None else None)


def layernorm_bwd(dy: Tensor, x: Tensor, mean: Tensor, rstd: Tensor,
                  gamma: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
    H = x.shape[-1]
    xf = _f(x).reshape(-1, H)
    g = _f(dy).reshape(-1, H)
    xhat = (xf - mean.reshape(-1, 1)) * rstd.reshape(-1, 1)
    dgamma = (g * xhat).sum(0)
    dbeta = g.sum(0)
    gg = g * _f(gamma)
    dx = rstd.reshape(-1, 1) * (gg - gg.mean(-1, keepdim=True) - xhat * (gg * xhat).mean(-1, keepdim=True))
    return dx.reshape(x.shape).to(dy.dtype), dgamma, dbeta


_M32 = 0xFFFFFFFF


def _mix32(x: Tensor) -> Tensor:
    """murmur3 finaliser on uint32 values held in int64 (bit-exact with the HIP kernels)."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x85EBCA6B) & _M32
    x = x ^ (x >> 13)
    x = (x * 0xC2B2AE35) & _M32
    return x ^ (x >> 16)


def _drop_threshold(p: float) -> int:
    return min(int(p * 4294967296.0), _M32)


def attention_keep(B: int, S: int, H: int, p: float, seed: int, device) -> Tensor:
    """[B,H,S(q),S(k)] keep mask of the attention-probability dropout (attention.hip keep_elem)."""
    q = torch.arange(S, device=device, dtype=torch.int64)
    bh = torch.arange(B * H, device=device, dtype=torch.int64)
    row_id = (bh[:, None] * S + q[None, :]) & _M32                      # [BH, S]
    a = _mix32(torch.full_like(row_id, seed & _M32) ^ ((row_id * 0x9E3779B1) & _M32))
    k = torch.arange(S, device=device, dtype=torch.int64)
    kk = (k * 0x85EBCA77 + 0x27D4EB2F) & _M32
    h = _mix32(a[:, :, None] ^ kk[None, None, :])
    return (h >= _drop_threshold(p)).reshape(B, H, S, S)


def dropout_keep(n: int, p: float, seed: int, device) -> Tensor:
    """flat keep mask of misc.hip dropout_kernel."""
    base = _mix32(torch.tensor(((seed & _M32) * 0x9E3779B1 + 0x7F4A7C15) & _M32, dtype=torch.int64))
    i = torch.arange(n, device=device, dtype=torch.int64)
    h = _mix32(base.to(device) ^ (((i & _M32) * 0x85EBCA77) & _M32))
    return h >= _drop_threshold(p)


def dropout_fwd(x: Tensor, p: float, seed: int) -> Tensor:
    if p <= 0.0:
        return x.clone()
    keep = dropout_keep(x.numel(), p, seed, x.device).reshape(x.shape)
    return (_f(x) * keep / (1.0 - p)).to(x.dtype)


def _split_qkv(qkv: Tensor, B: int, S: int, H: int):
    x = _f(qkv).reshape(B, S, 3, H, -1)
    return (x[:, :, 0].transpose(1, 2), x[:, :, 1].transpose(1, 2), x[:, :, 2].transpose(1, 2))


def attention_fwd(qkv: Tensor, B: int, S: int, H: int, mask: Optional[Tensor], scale: float,
                  p_drop: float = 0.0, seed: int = 0) -> Tuple[Tensor, Tensor]:
    """Packed layout of attention.hip: qkv [B*S, 3*H*D] -> (o [B*S, H*D], lse [B,H,S])."""
    q, k, v = _split_qkv(qkv, B, S, H)
    s = torch.einsum("bhqd,bhkd->bhqk", q, k) * scale
    if mask is not None:
        s = s + _f(mask).reshape(B, 1, 1, S)
    lse = torch.logsumexp(s, dim=-1)
    p = torch.exp(s - lse[..., None])
    if p_drop > 0.0:
        p = p * attention_keep(B, S, H, p_drop, seed, qkv.device) / (1.0 - p_drop)
    o = torch.einsum("bhqk,bhkd->bhqd", p, v)
    return o.transpose(1, 2).reshape(B * S, -1).to(qkv.dtype), lse


def attention_bwd(do: Tensor, qkv: Tensor, o: Tensor, lse: Tensor, B: int, S: int, H: int,
                  mask: Optional[Tensor], scale: float, p_drop: float = 0.0,
                  seed: int = 0) -> Tensor:
    q, k, v = _split_qkv(qkv, B, S, H)
    D = q.shape[-1]
    s = torch.einsum("bhqd,bhkd->bhqk", q, k) * scale
    if mask is not None:
        s = s + _f(mask).reshape(B, 1, 1, S)
    p = torch.exp(s - lse[..., None])
    dof = _f(do).reshape(B, S, H, D).transpose(1, 2)
    of = _f(o).reshape(B, S, H, D).transpose(1, 2)
    keep = None
    if p_drop > 0.0:
        keep = attention_keep(B, S, H, p_drop, seed, qkv.device) / (1.0 - p_drop)
    pd = p if keep is None else p * keep
    dv = torch.einsum("bhqk,bhqd->bhkd", pd, dof)
    dp = torch.einsum("bhqd,bhkd->bhqk", dof, v)
    if keep is not None:
        dp = dp * keep
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta) * scale
    dq = torch.einsum("bhqk,bhkd->bhqd", ds, k)
    dk = torch.einsum("bhqk,bhqd->bhkd", ds, q)
    out = torch.stack([t.transpose(1, 2) for t in (dq, dk, dv)], dim=2)  # [B,S,3,H,D]
    return out.reshape(B * S, 3 * H * D).to(qkv.dtype)


def embedding_bwd(dy: Tensor, idx: Tensor, num_rows: int) -> Tensor:
    H = dy.shape[-1]
    src = _f(dy.reshape(-1, H))
    out = torch.zeros(num_rows, H, dtype=src.dtype, device=dy.device)
    out.index_add_(0, idx.reshape(-1).long(), src)
    return out


def gelu_fwd(x: Tensor) -> Tensor:
    return F.gelu(_f(x)).to(x.dtype)


def gelu_bwd(dy: Tensor, x: Tensor) -> Tensor:
    xf = _f(x)
    cdf = 0.5 * (1.0 + torch.erf(xf / math.sqrt(2.0)))
    pdf = torch.exp(-0.5 * xf * xf) / math.sqrt(2.0 * math.pi)
    return (_f(dy) * (cdf + xf * pdf)).to(dy.dtype)


# ----------------------------------------------------------------------------- vision.hip
def act_fn(t: Tensor, act: str) -> Tensor:
    if act == "relu":
        return torch.relu(t)
    if act == "relu6":
        return t.clamp(0.0, 6.0)
    return t


def act_keep(z: Tensor, act: str) -> Optional[Tensor]:
    """Where the activation passes gradient, judged from its OUTPUT z like the kernels do
    (relu: z > 0; relu6: 0 < z < 6)."""
    if act == "relu":
        return z > 0
    if act == "relu6":
        return (z > 0) & (z < 6)
    return None


def _masked(dy: Tensor, z: Optional[Tensor], act: str) -> Tensor:
    g = _f(dy)
    keep = None if z is None else act_keep(_f(z), act)
    return g if keep is None else g * keep


def gconv_fwd(x: Tensor, w: Tensor, stride, pad, groups: int, bias: Optional[Tensor] = None,
              act: str = "none") -> Tensor:
    """y = act(conv(x, w, groups) + bias); x NHWC, w [Co, KH, KW, Ci/groups]; stride/pad (h, w)."""
    y = F.conv2d(_f(_nchw(x)), _f(_w_oihw(w)), None if bias is None else _f(bias),
                 stride=tuple(stride), padding=tuple(pad), groups=groups)
    return act_fn(_nhwc(y), act).to(x.dtype)


def gconv_dgrad(dy: Tensor, w: Tensor, x_shape, stride, pad, groups: int,
                z: Optional[Tensor] = None, act: str = "none") -> Tensor:
    N, H, W, Ci = x_shape
    g = _masked(dy, z, act)
    dx = torch.nn.grad.conv2d_input((N, Ci, H, W), _f(_w_oihw(w)), _nchw(g), stride=tuple(stride),
                                    padding=tuple(pad), groups=groups)
    return _nhwc(dx).to(dy.dtype)


def gconv_wgrad(dy: Tensor, x: Tensor, kh: int, kw: int, stride, pad, groups: int,
                z: Optional[Tensor] = None, act: str = "none") -> Tuple[Tensor, Tensor]:
    """(dw [Co, KH, KW, Ci/groups], db [Co]) in fp32 (fp64 inputs stay fp64)."""
    g = _masked(dy, z, act)
    Co, Ci = dy.shape[-1], x.shape[-1]
    dw = torch.nn.grad.conv2d_weight(_f(_nchw(x)), (Co, Ci // groups, kh, kw), _nchw(g),
                                     stride=tuple(stride), padding=tuple(pad), groups=groups)
    return dw.permute(0, 2, 3, 1).contiguous(), g.reshape(-1, Co).sum(0)


def chan_stats(y: Tensor, shift: Tensor) -> Tuple[Tensor, Tensor]:
    """Shifted per-channel sums Σ(y - shift), Σ(y - shift)² ([1, C] each)."""
    C = y.shape[-1]
    d = _f(y).reshape(-1, C) - _f(shift)[None, :]
    return d.sum(0, keepdim=True), (d * d).sum(0, keepdim=True)


def affine_act(y: Tensor, scale: Tensor, bias: Tensor, act: str = "none") -> Tensor:
    return act_fn(_f(y) * scale + bias, act).to(y.dtype)


def bn_generic_bwd_reduce(dz: Tensor, z: Optional[Tensor], y: Tensor, mean: Tensor,
                          invstd: Tensor, act: str = "none") -> Tuple[Tensor, Tensor]:
    """Σg and Σg·x̂ per channel, g = dz·act'(z), x̂ = (y - mean)·invstd."""
    C = y.shape[-1]
    g = _masked(dz, z, act).reshape(-1, C)
    xhat = (_f(y).reshape(-1, C) - mean) * invstd
    return g.sum(0), (g * xhat).sum(0)


def bn_generic_bwd_apply(dz: Tensor, z: Optional[Tensor], y: Tensor, mean: Tensor,
                         invstd: Tensor, gamma: Tensor, sum_g: Optional[Tensor],
                         sum_gx: Optional[Tensor], count: int, act: str = "none") -> Tensor:
    """dy = γ·invstd·(g − Σg/n − x̂·Σgx̂/n); without sums (eval-mode BN) dy = γ·invstd·g."""
    shp = y.shape
    C = shp[-1]
    g = _masked(dz, z, act).reshape(-1, C)
    if sum_g is None:
        dy = (_f(gamma) * invstd) * g
    else:
        xhat = (_f(y).reshape(-1, C) - mean) * invstd
        dy = (_f(gamma) * invstd) * (g - sum_g / count - xhat * (sum_gx / count))
    return dy.reshape(shp).to(dz.dtype)


def avgpool2d_fwd(x: Tensor, k: int, stride: int, pad: int) -> Tensor:
    return _nhwc(F.avg_pool2d(_f(_nchw(x)), k, stride, pad)).to(x.dtype)


def avgpool2d_bwd(dy: Tensor, x_shape, k: int, stride: int, pad: int) -> Tensor:
    N, H, W, C = x_shape
    with torch.enable_grad():
        xz = torch.zeros(N, C, H, W, dtype=_f(dy).dtype, device=dy.device, requires_grad=True)
        yz = F.avg_pool2d(xz, k, stride, pad)
        (g,) = torch.autograd.grad(yz, xz, _f(_nchw(dy)).contiguous())
    return _nhwc(g).to(dy.dtype)


def synthetic_images(indices: Tensor, num_classes: int, shape, seed: int,
                     dtype=torch.float32) -> Tuple[Tensor, Tensor]:
    """Deterministic, *learnable* synthetic NHWC images: label = hash(index) % classes,
    image = class template + unit gaussian noise keyed by (seed, index)."""
    N = indices.numel()
    H, W, C = shape
    idx = indices.long()
    labels = ((idx * 2654435761 + seed * 97) % 2147483647) % num_classes
    g = torch.Generator(device=indices.device)
    g.manual_seed(seed)
    templates = torch.randn(num_classes, H, W, C, generator=g, device=indices.device)
    noise = torch.empty(N, H, W, C, device=indices.device)
    for i in range(N):
        gi = torch.Generator(device=indices.device)
        gi.manual_seed(int(seed) * 7919 + int(idx[i]))
        noise[i] = torch.randn(H, W, C, generator=gi, device=indices.device)
    x = 0.5 * templates[labels] + noise
    return x.to(dtype), labels


def bn_relu_fold(y: Tensor, scale: Tensor, bias: Tensor) -> Tensor:
    """The operand a folded input BatchNorm hands its consumer conv: relu(y*scale + bias) per
    channel (NHWC), in y's dtype — the values bn_act_fwd would have stored."""
    return torch.relu(y.float() * scale.float() + bias.float()).to(y.dtype)
