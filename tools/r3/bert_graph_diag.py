#!/usr/bin/env python3
"""Where does a hipGraph-replayed BERT step differ from the eager one?  Per-parameter max |diff|
graph-vs-eager and eager-vs-eager, with and without dropout, after 1 warm-up + 3 replays."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(dropout: bool, replays: int = 3):
    from mipipe.models import create_model
    from mipipe.optim import AdamW
    from mipipe.train.graph import GraphedStep
    kw = {} if dropout else {"hidden_dropout_prob": 0.0, "attention_probs_dropout_prob": 0.0}
    torch.manual_seed(0)
    a = create_model("bert_tiny", **kw).cuda()
    b, c = copy.deepcopy(a), copy.deepcopy(a)
    opts = [AdamW(m.parameters(), lr=1e-3, weight_decay=0.01) for m in (a, b, c)]
    B, S, P, V = 8, 128, 20, a.config.vocab_size
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    ids = torch.randint(0, V, (B, S), device="cuda", generator=g)
    am = torch.ones(B, S, device="cuda", dtype=torch.int64)
    pos = torch.stack([torch.randperm(S, device="cuda", generator=g)[:P] for _ in range(B)])
    labels = torch.randint(0, V, (B, P), device="cuda", generator=g)
    batch = (ids, am, pos, labels)

    def fn(m, o):
        def step(i_, a_, p_, l_):
            o.zero_grad()
            loss = m(i_, a_, masked_positions=p_, labels=l_)
            loss.backward()
            o.step()
            return loss
        return step

    la = [fn(a, opts[0])(*batch).item() for _ in range(1 + replays)]
    lc = [fn(c, opts[2])(*batch).item() for _ in range(1 + replays)]
    gs = GraphedStep(fn(b, opts[1]), batch, warmup=1, inputs=[batch])
    lb = [gs.warmup_loss.item()] + [gs.replay(0).item() for _ in range(replays)]
    torch.cuda.synchronize()
    print(f"dropout={dropout} losses eager {la}\n  graph {lb}\n  eager2 {lc}")
    for (n, p), (_, q), (_, r) in zip(a.named_parameters(), b.named_parameters(), c.named_parameters()):
        d_pq = (p - q).abs().max().item()
        d_pr = (p - r).abs().max().item()
        flag = "  <<<" if d_pq > 3 * d_pr + 1e-5 else ""
        print(f"  {n:60s} graph {d_pq:.3e} eager2 {d_pr:.3e}{flag}")
    print(f"  counters: eager {int(a._step_dev.item())}/{opts[0].sync_step()} "
          f"graph {int(b._step_dev.item())}/{opts[1].sync_step()}")


if __name__ == "__main__":
    run(True)
    run(False)
