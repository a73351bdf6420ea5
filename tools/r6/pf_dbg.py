import copy
import torch
from mipipe.ops import prefetch
import mipipe.ops.functional as F
from mipipe.models import create_model
from mipipe.ops.determinism import deterministic
from mipipe.optim import AdamW
import tests.test_prefetch_gpu as T
seqs=[[]]
orig=prefetch.before_weight_gemm
def hook(w, also=None):
    seqs[-1].append((w.data_ptr(), tuple(w.shape)))
    orig(w, also)
    print("  gemm", len(seqs[-1]), prefetch._S.armed, prefetch._S.recording, len(prefetch._S.order), prefetch._S.cursor, flush=True)
F._prefetch.before_weight_gemm = hook
with deterministic(True):
    torch.manual_seed(0)
    a = create_model("bert_tiny").cuda()
    b, c = copy.deepcopy(a), copy.deepcopy(a)
    opts = [AdamW(m.parameters(), lr=1e-3, weight_decay=0.01) for m in (a, b, c)]
    batch = T._batch(a.config.vocab_size)
    prefetch.reset()
    prefetch._MODE = "1"
    for s in range(3):
        seqs.append([])
        print("step", s, flush=True)
        T._step_fn(c, opts[2])(*batch)
    for i,(x,y) in enumerate(zip(seqs[1],seqs[2])):
        if x!=y: print("diff", i, x, y)
