"""Single-process multi-GPU data parallelism (reference path (d), task.py:201-208).

In the reference this path is effectively dead (it later crashes in DistributedSampler
without a process group); it is kept for API parity.  Replicas are produced by
``torch.nn.parallel.replicate``; mipipe layers fetch their compute-dtype weight on the
replica's device, so the HIP kernels run on every GPU.  With one visible GPU it is a plain
pass-through, the common case on a 1-GPU box.
"""
from __future__ import annotations

import torch
import torch.nn as tnn

__all__ = ["DataParallel"]


class DataParallel(tnn.DataParallel):
    def forward(self, *inputs, **kwargs):
        if not self.device_ids or len(self.device_ids) == 1:
            return self.module(*inputs, **kwargs)
        return super().forward(*inputs, **kwargs)
