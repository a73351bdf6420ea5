"""Attribute the stock ATen kernels in a BERT-base MLM training step to their Python call sites."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import profile, ProfilerActivity
from mipipe.models import create_model
from mipipe.optim import AdamW
dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = create_model("bert_base").to(dev)
m.compute_dtype = torch.bfloat16
opt = AdamW(m.parameters(), lr=1e-4, weight_decay=0.01)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
S = int(sys.argv[2]) if len(sys.argv) > 2 else 128
P, V = (20 if S == 128 else round(0.15 * S)), 30522
ids = torch.randint(0, V, (B, S), device=dev)
am = torch.ones(B, S, device=dev, dtype=torch.int64)
pos = torch.stack([torch.randperm(S, device=dev)[:P] for _ in range(B)])
lab = torch.randint(0, V, (B, P), device=dev)
def step():
    opt.zero_grad()
    loss = m(ids, am, masked_positions=pos, labels=lab)
    loss.backward()
    opt.step()
for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    step()
    torch.cuda.synchronize()
for ev in sorted(prof.key_averages(group_by_stack_n=6), key=lambda e: -e.device_time_total):
    if ev.key.startswith("aten::") and ev.device_time_total > 0:
        print(f"{ev.key:16s} n={ev.count:4d} dev_us={ev.device_time_total:9.1f}")
        for fr in ev.stack[:6]:
            print("      ", fr)
