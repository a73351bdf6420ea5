"""BERT MLM on CPU (reference-kernel path): fp64 parity with the stock torch.nn/SDPA model,
HuggingFace-style state_dict interchange, hash-dropout determinism and the packed attention
contract of attention.hip."""
import math

import pytest
import torch

from mipipe.models import create_model, model_names
from mipipe.models.reference import ref_bert
from mipipe.ops import _ref
from mipipe.ops import functional as MF


def _tiny_pair(dropout=0.0):
    torch.manual_seed(0)
    m = create_model("bert_tiny", hidden_dropout_prob=dropout,
                     attention_probs_dropout_prob=dropout).double()
    m.compute_dtype = torch.float64
    r = ref_bert("bert_tiny", hidden_dropout_prob=dropout,
                 attention_probs_dropout_prob=dropout).double()
    r.load_state_dict(m.state_dict(), strict=True)
    return m, r


def test_registry_has_bert():
    assert {"bert", "bert_base", "bert_tiny"} <= set(model_names())


def test_bert_fp64_parity_with_stock_model():
    m, r = _tiny_pair()
    B, S = 2, 16
    ids = torch.randint(0, 30522, (B, S))
    am = torch.ones(B, S)
    am[1, 11:] = 0
    pos = torch.stack([torch.randperm(S)[:3] for _ in range(B)])
    labels = torch.randint(0, 30522, (B * 3,))
    lo, lr = m(ids, am, masked_positions=pos), r(ids, am, masked_positions=pos)
    assert lo.shape == lr.shape == (B * 3, 30522)
    assert (lo - lr).abs().max() < 1e-10
    loss = m(ids, am, masked_positions=pos, labels=labels)
    loss_r = r.loss(lr, labels)
    assert abs(loss.item() - loss_r.item()) < 1e-10
    loss.backward()
    loss_r.backward()
    rp = dict(r.named_parameters())
    for n, p in m.named_parameters():
        if ".qkv." in n:
            kind = n.rsplit(".", 1)[1]
            pre = n[: -len("qkv." + kind)]
            g = torch.cat([rp[f"{pre}{x}.{kind}"].grad for x in ("query", "key", "value")])
        else:
            g = rp[n].grad
        assert (p.grad - g).abs().max() <= 1e-6 * (g.abs().max() + 1e-30), n


def test_bert_state_dict_is_hf_keyed_and_roundtrips():
    m, r = _tiny_pair()
    sd = m.state_dict()
    assert "bert.encoder.layer.0.attention.self.query.weight" in sd
    assert "cls.predictions.decoder.weight" in sd
    assert not any(".qkv." in k for k in sd)
    assert set(sd) == set(r.state_dict())
    m2 = create_model("bert_tiny")
    m2.load_state_dict(r.state_dict(), strict=True)
    for (n, a), (_, b) in zip(m.named_parameters(), m2.named_parameters()):
        assert torch.equal(a.float(), b.float()), n


def test_hash_dropout_regenerates_mask_in_backward():
    x = torch.randn(4, 64, dtype=torch.float64, requires_grad=True)
    y = MF.dropout(x, 0.25, seed=123)
    y2 = MF.dropout(x, 0.25, seed=123)
    assert torch.equal(y, y2)
    keep = y != 0
    frac = keep.float().mean().item()
    assert 0.6 < frac < 0.9
    assert torch.allclose(y[keep], x[keep] / 0.75)
    y.sum().backward()
    assert torch.equal(x.grad != 0, keep)
    assert not torch.equal(MF.dropout(x, 0.25, seed=124), y)


@pytest.mark.parametrize("p_drop", [0.0, 0.2])
def test_packed_attention_matches_naive(p_drop):
    torch.manual_seed(0)
    B, S, H, D = 2, 10, 3, 64
    qkv = torch.randn(B * S, 3 * H * D, dtype=torch.float64, requires_grad=True)
    mask = torch.zeros(B, S, dtype=torch.float64)
    mask[0, 7:] = -10000.0
    o = MF.attention(qkv, B, S, H, mask, p_drop=p_drop, seed=5)
    x = qkv.reshape(B, S, 3, H, D)
    q, k, v = (x[:, :, i].transpose(1, 2) for i in range(3))
    s = q @ k.transpose(-1, -2) / math.sqrt(D) + mask[:, None, None, :]
    p = s.softmax(-1)
    if p_drop:
        p = p * _ref.attention_keep(B, S, H, p_drop, 5, "cpu") / (1 - p_drop)
    ref = (p @ v).transpose(1, 2).reshape(B * S, H * D)
    assert (o - ref).abs().max() < 1e-10
    g = torch.randn_like(o)
    (dq,) = torch.autograd.grad(o, qkv, g)
    (dr,) = torch.autograd.grad(ref, qkv, g)
    assert (dq - dr).abs().max() < 1e-9


def test_bert_trains_on_cpu():
    torch.manual_seed(0)
    m = create_model("bert_tiny")
    from mipipe.optim import AdamW
    opt = AdamW(m.parameters(), lr=1e-3, weight_decay=0.01)
    B, S = 4, 16
    ids = torch.randint(0, 1000, (B, S))
    pos = torch.stack([torch.randperm(S)[:3] for _ in range(B)])
    labels = torch.gather(ids, 1, pos)
    losses = []
    for _ in range(8):
        opt.zero_grad()
        loss = m(ids, masked_positions=pos, labels=labels)
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert losses[-1] < losses[0]


def test_padded_decoder_views_match_copy_path_cpu():
    """Flat-space padded decoder views (optimizer present) vs the padded-copy path: same loss
    and gradients; the reserved pad rows stay zero through optimizer steps."""
    from mipipe.optim import AdamW
    from mipipe.optim.flat import flat_space_for
    torch.manual_seed(0)
    kw = dict(hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m1, m2 = create_model("bert_tiny", **kw), create_model("bert_tiny", **kw)
    m2.load_state_dict(m1.state_dict())
    opt = AdamW(m1.parameters(), lr=1e-3, weight_decay=0.01)
    fs = flat_space_for(m1.cls.predictions.bias)
    assert fs.padded_rows(m1.bert.embeddings.word_embeddings.weight) == 30528
    B, S = 2, 16
    ids = torch.randint(0, 30522, (B, S))
    pos = torch.stack([torch.randperm(S)[:3] for _ in range(B)])
    labels = torch.randint(0, 30522, (B * 3,))
    opt.zero_grad()
    l1 = m1(ids, masked_positions=pos, labels=labels)
    l2 = m2(ids, masked_positions=pos, labels=labels)
    assert abs(l1.item() - l2.item()) < 1e-5
    l1.backward()
    l2.backward()
    for (n, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.allclose(p1.grad, p2.grad, atol=1e-6, rtol=1e-4), n
    opt.step()
    for p in (m1.bert.embeddings.word_embeddings.weight, m1.cls.predictions.bias):
        assert torch.count_nonzero(fs.padded_view(fs.flat, p)[p.shape[0]:]) == 0
