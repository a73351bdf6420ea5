"""Temporary: fused dgrad epilogue timing under experiment knobs (bit0 skip reduction/atomics,
bit1 constant BN params, bit2 skip per-element BN math)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from mipipe.ops._native import native  # noqa: E402
from tools.r2.dgrad_epi_probe import timed  # noqa: E402

nat = native()
dev = torch.device("cuda")
R = nat.STAT_REPLICAS
for name, (N, H, Co, Ci) in {"l1.conv1": (256, 56, 64, 256), "l1.conv3": (256, 56, 256, 64),
                             "l3.conv1": (256, 14, 256, 1024)}.items():
    bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)  # noqa: E731
    dy = bf(N, H, H, Co)
    w = (torch.randn(Co, 1, 1, Ci, device=dev) * 0.05).to(torch.bfloat16)
    y, add = bf(N, H, H, Ci), bf(N, H, H, Ci)
    mean, invstd = torch.zeros(Ci, device=dev), torch.ones(Ci, device=dev)
    scale, bias = torch.ones(Ci, device=dev), torch.zeros(Ci, device=dev)
    rep = torch.zeros(3, R, Ci, device=dev)
    shp = [N, H, H, Ci]
    for cfg in (9, 7, 2):
        row = {"shape": name, "cfg": cfg,
               "addend": round(timed(lambda: nat.conv_dgrad(dy, w, shp, 1, 0, add, cfg=cfg)), 1)}
        for knob in (0, 1, 2, 4, 3, 7):
            nat.set_epi_knob(knob)
            row[f"bn_y_k{knob}"] = round(timed(lambda: nat.conv_dgrad(
                dy, w, shp, 1, 0, None, y, mean, invstd, scale, bias, rep, cfg=cfg)), 1)
        nat.set_epi_knob(0)
        print(json.dumps(row), flush=True)
