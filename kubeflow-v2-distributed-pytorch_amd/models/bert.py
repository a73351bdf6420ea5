"""BERT-base masked-LM on mipipe's fused kernels (BASELINE config 4).

The reference trains torchvision CNNs only (task.py:50-52, 165-171); BASELINE.json adds a
"BERT-base MLM DDP" config whose kernel list SURVEY.md §2.5 gives: QKV / output / FFN GEMMs with
bias and GELU epilogues, LayerNorm fwd/bwd, flash-style attention, embedding gather +
scatter-add backward, the MLM head GEMM + cross-entropy over 30522 classes, dropout and fused
AdamW.  Every one of those runs on a mipipe HIP kernel here:

* one fused QKV projection GEMM per layer; its [tokens, 3*768] output is consumed in place by
  the attention kernel (attention.hip) and the attention output feeds the output projection
  without any head transpose;
* post-LN residual adds are fused into the LayerNorm kernel (``LN(x + residual)``);
* dropout masks are hashed from (seed, element) and regenerated in the backward;
* the MLM head runs only on the masked positions (``masked_positions``, NVIDIA/Megatron
  style) — the loss and gradients equal the dense head's, which spends ~85 % of its FLOPs on
  ignored (-100) tokens.

``state_dict`` keys follow HuggingFace ``BertForMaskedLM`` (``bert.embeddings.*``,
``bert.encoder.layer.N.attention.self.{query,key,value}.*`` ...): the fused QKV parameter is
split / merged by state-dict hooks, so checkpoints interchange with the stock model in
:mod:`mipipe.models.reference`.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn as tnn

from mipipe import nn as mnn
from mipipe.ops import functional as MF
from mipipe.ops import kernels as K

from . import register_model


@dataclass
class BertConfig:
    vocab_size: int = 30522
    hidden_size: int = 768
    num_hidden_layers: int = 12
    num_attention_heads: int = 12
    intermediate_size: int = 3072
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    hidden_dropout_prob: float = 0.1
    attention_probs_dropout_prob: float = 0.1
    initializer_range: float = 0.02


def _seed(base: int, step: int, site: int) -> int:
    return (base * 0x9E3779B1 + step * 0x85EBCA77 + site * 0xC2B2AE35 + 0x165667B1) & 0xFFFFFFFF


class _Embeddings(tnn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.word_embeddings = mnn.Embedding(c.vocab_size, c.hidden_size)
        self.position_embeddings = mnn.Embedding(c.max_position_embeddings, c.hidden_size)
        self.token_type_embeddings = mnn.Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = mnn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)


class _SelfAttention(tnn.Module):
    """Holds the fused ``qkv`` projection; exposes HF's query/key/value keys via hooks."""

    def __init__(self, c: BertConfig):
        super().__init__()
        self.qkv = mnn.Linear(c.hidden_size, 3 * c.hidden_size)


class _Dense(tnn.Module):
    def __init__(self, cin: int, cout: int, eps: Optional[float] = None):
        super().__init__()
        self.dense = mnn.Linear(cin, cout)
        if eps is not None:
            self.LayerNorm = mnn.LayerNorm(cout, eps=eps)


class _Attention(tnn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.self = _SelfAttention(c)
        self.output = _Dense(c.hidden_size, c.hidden_size, c.layer_norm_eps)


class BertLayer(tnn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.attention = _Attention(c)
        self.intermediate = _Dense(c.hidden_size, c.intermediate_size)
        self.output = _Dense(c.intermediate_size, c.hidden_size, c.layer_norm_eps)
        self.heads = c.num_attention_heads
        self.p_hidden = c.hidden_dropout_prob
        self.p_attn = c.attention_probs_dropout_prob

    def forward(self, h: torch.Tensor, B: int, S: int, mask: Optional[torch.Tensor],
                seeds) -> torch.Tensor:
        train = self.training
        # h and h1 each feed a projection AND a post-LN residual: the LayerNorm backward hands
        # the residual gradient to the projection, whose data-grad GEMM adds it (no extra add)
        s_h, s_h1 = MF.ResidualSlot(), MF.ResidualSlot()
        # and each post-LN kernel's backward sums its branch's bias gradient (no colsum pass)
        s_b1, s_b2 = MF.BiasGradSlot(), MF.BiasGradSlot()
        qkv = self.attention.self.qkv(h, res_take=s_h)
        ctx = MF.attention(qkv, B, S, self.heads, mask, p_drop=self.p_attn if train else 0.0,
                           seed=seeds[0])
        a = self.attention.output.dense(ctx, bias_slot=s_b1)
        # hidden dropout fused into the post-LN residual kernels (same mask as MF.dropout)
        p = self.p_hidden if train else 0.0
        h1 = self.attention.output.LayerNorm(a, residual=h, res_give=s_h, dropout_p=p,
                                             dropout_seed=seeds[1], bias_slot=s_b1)
        f = self.intermediate.dense(h1, act="gelu", res_take=s_h1)
        f2 = self.output.dense(f, bias_slot=s_b2)
        return self.output.LayerNorm(f2, residual=h1, res_give=s_h1, dropout_p=p,
                                     dropout_seed=seeds[2], bias_slot=s_b2)


class _Encoder(tnn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.layer = tnn.ModuleList([BertLayer(c) for _ in range(c.num_hidden_layers)])


class _BertModel(tnn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.embeddings = _Embeddings(c)
        self.encoder = _Encoder(c)


class _Transform(tnn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.dense = mnn.Linear(c.hidden_size, c.hidden_size)
        self.LayerNorm = mnn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)


class _Predictions(tnn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.transform = _Transform(c)
        self.bias = tnn.Parameter(torch.zeros(c.vocab_size))


class _Cls(tnn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.predictions = _Predictions(c)


class BertForMaskedLM(tnn.Module):
    """``forward(input_ids, attention_mask=None, token_type_ids=None, masked_positions=None)``
    -> MLM logits ``[B*P, V]`` for the masked positions (or ``[B*S, V]`` for all tokens).
    ``loss(logits, labels)`` = mean cross-entropy (labels -100 ignored)."""

    # dropout seeds take their per-step part from a device counter on the GPU (graph-replayable)
    device_seeds = True

    def __init__(self, config: Optional[BertConfig] = None, compute_dtype=None, seed: int = 0,
                 **kw):
        super().__init__()
        c = config or BertConfig(**{k: v for k, v in kw.items() if hasattr(BertConfig, k)})
        self.config = c
        self.compute_dtype = compute_dtype
        self.bert = _BertModel(c)
        self.cls = _Cls(c)
        self.seed = seed
        self.rank_override: Optional[int] = None  # dropout-seed rank (bench --emulate-ranks)
        self._step = 0
        self._step_dev: Optional[torch.Tensor] = None  # device step counter (dropout seeds)
        self._vpad = (-c.vocab_size) % 64  # decoder N padded to the GEMM's 64-wide tiles
        self._init_weights()
        # the tied decoder's weight-gradient GEMM runs before the embedding lookup's scatter in
        # the backward: only the latter may report the shared gradient complete (DDP buckets)
        # — unless DDP exchanges the lookup part sparsely (parallel/ddp.py, a sink on the
        # weight): then the decoder's dense part is complete at the START of the backward and
        # DDP puts the weight's flat slot first, into the first gradient bucket
        self.bert.embeddings.word_embeddings.weight._mipipe_tied_later = True
        if self._vpad:
            # the flat parameter space (mipipe.optim) reserves zero rows behind the tied
            # decoder weight / bias: the padded decoder operand is a view, not a per-step copy
            vp = c.vocab_size + self._vpad
            self.bert.embeddings.word_embeddings.weight._mipipe_pad_rows = vp
            self.cls.predictions.bias._mipipe_pad_rows = vp
        self._register_state_dict_hook(_split_qkv_hook)
        self._register_load_state_dict_pre_hook(_merge_qkv_hook, with_module=True)

    # HF BertPreTrainedModel._init_weights
    def _init_weights(self):
        std = self.config.initializer_range
        for m in self.modules():
            if isinstance(m, tnn.Linear):
                tnn.init.normal_(m.weight, 0.0, std)
                if m.bias is not None:
                    tnn.init.zeros_(m.bias)
            elif isinstance(m, tnn.Embedding):
                tnn.init.normal_(m.weight, 0.0, std)
            elif isinstance(m, tnn.LayerNorm):
                tnn.init.ones_(m.weight)
                tnn.init.zeros_(m.bias)

    def activation_dtype(self, ref: torch.Tensor) -> torch.dtype:
        if self.compute_dtype is not None:
            return self.compute_dtype
        return torch.bfloat16 if ref.is_cuda else torch.float32

    def forward(self, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None,
                token_type_ids: Optional[torch.Tensor] = None,
                masked_positions: Optional[torch.Tensor] = None,
                labels: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Returns the MLM loss when ``labels`` is given (cross-entropy straight on the
        tile-padded logits, the pad columns excluded), else the logits."""
        c = self.config
        B, S = input_ids.shape
        dt = self.activation_dtype(input_ids)
        emb = self.bert.embeddings
        if self.training:
            self._step += 1
        rank = torch.distributed.get_rank() if torch.distributed.is_initialized() else 0
        if self.rank_override is not None:
            rank = self.rank_override
        base = (self.seed + 7919 * rank) & 0xFFFFFFFF
        # On the GPU the per-step part of every dropout seed is a device counter advanced here by
        # a device op, so a hipGraph-captured step draws fresh masks on every replay (the host
        # counter self._step would be frozen at capture).
        # The counter starts at the host step (so a resumed run, whose _step the checkpoint
        # restores, continues the mask sequence), and each forward hands its kernels a SNAPSHOT
        # of it: the backward regenerates its masks from the value this forward used even if
        # another training forward advances the counter before this backward runs.
        sdev = None
        if self.training and input_ids.is_cuda:
            if self._step_dev is None or self._step_dev.device != input_ids.device:
                self._step_dev = torch.full((1,), self._step - 1, dtype=torch.int32,
                                            device=input_ids.device)
            self._step_dev.add_(1)
            sdev = self._step_dev.clone()

        def seed_at(site: int):
            if sdev is not None:
                return K.DevSeed(_seed(base, 0, site), sdev)
            return _seed(base, self._step, site)

        ids = input_ids.reshape(-1)
        # position / default token-type ids per batch shape, made once (3 fewer launches a step)
        key = (B, S, ids.device)
        pc = getattr(self, "_ids_cache", None)
        if pc is None or pc[0] != key:
            pc = (key, torch.arange(S, device=ids.device).repeat(B), torch.zeros_like(ids))
            self._ids_cache = pc
        pos = pc[1]
        tt = pc[2] if token_type_ids is None else token_type_ids.reshape(-1)
        w = emb.word_embeddings(ids, dt)
        pt = emb.position_embeddings(pos, dt) + emb.token_type_embeddings(tt, dt)
        h = emb.LayerNorm(w, residual=pt)
        h = MF.dropout(h, c.hidden_dropout_prob, seed_at(0), self.training)
        mask = None
        if attention_mask is not None:
            mask = (1.0 - attention_mask.float()) * -10000.0  # HF extended attention mask
        for i, layer in enumerate(self.bert.encoder.layer):
            seeds = [seed_at(3 * i + j + 1) for j in range(3)]
            h = layer(h, B, S, mask, seeds)
        if masked_positions is not None:
            P = masked_positions.shape[1]
            rows = (masked_positions + torch.arange(B, device=h.device)[:, None] * S).reshape(-1)
            h = h.index_select(0, rows)
        pr = self.cls.predictions
        t = pr.transform.dense(h, act="gelu")
        t = pr.transform.LayerNorm(t)
        wd, bias_c = self._decoder_operands(dt)  # tied decoder, vocabulary tile-padded
        logits = MF.linear(t, emb.word_embeddings.weight, wd, pr.bias, "none", bias_c=bias_c)
        if labels is not None:
            return MF.cross_entropy(logits, labels.reshape(-1), ignore_index=-100,
                                    valid_cols=c.vocab_size)
        return logits[:, : c.vocab_size] if self._vpad else logits

    def _decoder_operands(self, dt: torch.dtype):
        """(decoder weight [Vp, H] in dtype dt, bias [Vp] fp32) with Vp = vocab rounded up to the
        GEMM tile width.  Pad rows / entries are zeros; the loss masks the pad columns.  Views of
        the flat parameter space's reserved pad rows when the optimizer built one (no copy),
        else a padded copy (evaluation without an optimizer, CPU)."""
        from mipipe.optim.flat import flat_space_for
        wte = self.bert.embeddings.word_embeddings
        bias = self.cls.predictions.bias
        if not self._vpad:
            return wte.compute_weight(dt), None
        fs = flat_space_for(wte.weight)
        if fs is not None and fs.padded_rows(wte.weight) and fs.padded_rows(bias) \
                and flat_space_for(bias) is fs:
            bias_c = fs.padded_view(fs.flat, bias)
            if fs.shadow is not None and fs.shadow.dtype == dt:
                fs.sync_shadow(wte.weight)
                return fs.padded_view(fs.shadow, wte.weight), bias_c
            if dt == torch.float32:
                return fs.padded_view(fs.flat, wte.weight), bias_c
        wd = wte.compute_weight(dt)
        wd = torch.cat([wd, wd.new_zeros(self._vpad, wd.shape[1])], 0)
        return wd, torch.cat([bias.detach(), bias.new_zeros(self._vpad)])

    def loss(self, logits: torch.Tensor, labels: torch.Tensor) -> torch.Tensor:
        return MF.cross_entropy(logits.contiguous(), labels.reshape(-1), ignore_index=-100)


def _split_qkv_hook(module, state_dict, prefix, local_metadata):
    for k in list(state_dict.keys()):
        if k.endswith("attention.self.qkv.weight") or k.endswith("attention.self.qkv.bias"):
            kind = k.rsplit(".", 1)[1]
            base = k[: -len(f"qkv.{kind}")]
            t = state_dict.pop(k)
            for name, part in zip(("query", "key", "value"), t.chunk(3, 0)):
                state_dict[f"{base}{name}.{kind}"] = part
        if k.endswith("cls.predictions.bias"):
            state_dict[k[: -len("bias")] + "decoder.bias"] = state_dict[k]
    if prefix + "bert.embeddings.word_embeddings.weight" in state_dict:
        state_dict[prefix + "cls.predictions.decoder.weight"] = \
            state_dict[prefix + "bert.embeddings.word_embeddings.weight"]
    for k in list(state_dict.keys()):
        if k.endswith("position_ids"):
            state_dict.pop(k)
    return state_dict


def _merge_qkv_hook(module, state_dict, prefix, local_metadata, strict, missing_keys,
                    unexpected_keys, error_msgs):
    for k in list(state_dict.keys()):
        for kind in ("weight", "bias"):
            if k.startswith(prefix) and k.endswith(f"attention.self.query.{kind}"):
                base = k[: -len(f"query.{kind}")]
                parts = [state_dict.pop(f"{base}{n}.{kind}") for n in ("query", "key", "value")]
                state_dict[f"{base}qkv.{kind}"] = torch.cat(parts, 0)
    for extra in ("cls.predictions.decoder.weight", "cls.predictions.decoder.bias",
                  "bert.embeddings.position_ids"):
        state_dict.pop(prefix + extra, None)


def bert_base(**kw) -> BertForMaskedLM:
    return BertForMaskedLM(**kw)


def bert_tiny(**kw) -> BertForMaskedLM:
    """2-layer, hidden 128 variant for tests."""
    cfg = BertConfig(hidden_size=128, num_hidden_layers=2, num_attention_heads=2,
                     intermediate_size=512, **{k: v for k, v in kw.items()
                                                if k in BertConfig.__dataclass_fields__})
    rest = {k: v for k, v in kw.items() if k not in BertConfig.__dataclass_fields__}
    return BertForMaskedLM(cfg, **rest)


register_model("bert_base", bert_base)
register_model("bert", bert_base)
register_model("bert_tiny", bert_tiny)
