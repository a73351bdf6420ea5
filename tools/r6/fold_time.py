"""Per-tile time of the folded-BN (BNIN) conv forward / weight-grad vs the plain kernels on the
ResNet-50 b256 conv3 shapes (python tools/r6/fold_time.py > out.jsonl)."""
import json

import torch

from mipipe.ops._native import native

SHAPES = [(256, 56, 56, 64, 256), (256, 28, 28, 128, 512), (256, 14, 14, 256, 1024),
          (256, 7, 7, 512, 2048)]


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    C = native()
    for N, H, W, Ci, Co in SHAPES:
        y = torch.randn(N, H, W, Ci, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Co, 1, 1, Ci, device="cuda") / Ci ** 0.5).to(torch.bfloat16)
        sc, bi = torch.rand(Ci, device="cuda") + 0.5, torch.randn(Ci, device="cuda") * 0.5
        sh = torch.zeros(Co, device="cuda")
        dy = torch.randn(N, H, W, Co, device="cuda").to(torch.bfloat16)
        for cfg in range(11):
            r = {"shape": [N, H, W, Ci, Co], "cfg": cfg,
                 "fwd_us": timeit(lambda: C.conv_fwd(y, w, 1, 0, sh, cfg=cfg)),
                 "fwd_bn_us": timeit(lambda: C.conv_fwd(y, w, 1, 0, sh, cfg=cfg, in_scale=sc,
                                                        in_bias=bi)),
                 "wgrad_us": timeit(lambda: C.conv_wgrad(dy, y, 1, 1, 1, 0, cfg=cfg)),
                 "wgrad_bn_us": timeit(lambda: C.conv_wgrad(dy, y, 1, 1, 1, 0, cfg=cfg,
                                                            in_scale=sc, in_bias=bi))}
            print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}),
                  flush=True)


if __name__ == "__main__":
    main()
