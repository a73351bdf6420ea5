"""Synthetic, learnable image datasets (no network on the MI355X node).

The reference downloads CIFAR-10 in every process (task.py:256-257, a race it admits in
task.py:254-255) and decodes/augments it in 8 CPU workers per rank (task.py:263).  Here data
is generated *on the device* from (seed, sample index): label = hash(index) mod classes,
image = 0.5·template[label] + N(0,1) noise, so a model can actually learn (accuracy rises
above chance, which the pipeline's ``baseline_accuracy`` gate uses) while no bytes cross
PCIe and no CPU worker is needed.  Values are normalised (zero-mean, ~unit variance), the
statistics ``transforms.Normalize`` produces for real data.

``SyntheticImageDataset`` is a map-style ``torch.utils.data.Dataset`` (CPU tensors, for
DataLoader use); ``DeviceBatchLoader`` yields whole batches generated on the GPU by a HIP
kernel (or ATen on CPU) for the indices a :class:`DistributedSampler` assigns to this rank.
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Sequence, Tuple

import torch

__all__ = ["SyntheticImageDataset", "DeviceBatchLoader", "synthetic_batch", "DATASET_SHAPES"]

# name -> (channels, height, width, classes, samples)
DATASET_SHAPES = {
    "cifar10": (3, 32, 32, 10, 10000),       # reference: CIFAR10(train=False) 10k images
    "mnist": (1, 28, 28, 10, 10000),
    "imagenet": (3, 224, 224, 1000, 1281167),
}

_M1 = 0x9E3779B1
_M2 = 0x85EBCA77
_M3 = 0xC2B2AE3D


def _mix32(x: torch.Tensor) -> torch.Tensor:
    """murmur3-style finalizer on int64 tensors holding 32-bit values."""
    x = x & 0xFFFFFFFF
    x = x ^ (x >> 16)
    x = (x * _M2) & 0xFFFFFFFF
    x = x ^ (x >> 13)
    x = (x * _M3) & 0xFFFFFFFF
    x = x ^ (x >> 16)
    return x


def _uniform(h: torch.Tensor) -> torch.Tensor:
    return ((h >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)


def synthetic_batch(indices: torch.Tensor, shape: Sequence[int], num_classes: int, seed: int,
                    dtype: torch.dtype = torch.float32) -> Tuple[torch.Tensor, torch.Tensor]:
    """NCHW images + int64 labels for ``indices`` (any device).  Uses the HIP kernel on GPU."""
    C, H, W = shape
    if indices.is_cuda:
        from mipipe.ops._native import native_available, native
        if native_available():
            return native().synthetic_batch(indices, C, H, W, num_classes, seed, dtype)
    idx = indices.to(torch.int64)
    labels = _mix32(idx * _M1 + seed * 7919 + 17) % num_classes
    n = idx.numel()
    P = C * H * W
    pos = torch.arange(P, device=indices.device, dtype=torch.int64)
    # template value per (class, pos)
    tkey = _mix32(labels[:, None] * 0x27D4EB2F + pos[None, :] * _M1 + seed * 31 + 1)
    t1 = _uniform(tkey)
    t2 = _uniform(_mix32(tkey + 0x165667B1))
    templ = torch.sqrt(-2.0 * torch.log(t1)) * torch.cos(6.283185307179586 * t2)
    nkey = _mix32(idx[:, None] * 0x632BE5AB + pos[None, :] * _M2 + seed * 131 + 7)
    u1 = _uniform(nkey)
    u2 = _uniform(_mix32(nkey + 0x27D4EB2F))
    noise = torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(6.283185307179586 * u2)
    x = (0.5 * templ + noise).reshape(n, C, H, W).to(dtype)
    return x, labels


class SyntheticImageDataset(torch.utils.data.Dataset):
    """Map-style dataset with torchvision-like ``(image CHW float, label int)`` items."""

    def __init__(self, name: str = "cifar10", length: Optional[int] = None, seed: int = 0,
                 shape: Optional[Sequence[int]] = None, num_classes: Optional[int] = None):
        C, H, W, K, N = DATASET_SHAPES[name]
        self.shape = tuple(shape) if shape is not None else (C, H, W)
        self.num_classes = num_classes or K
        self.length = length if length is not None else N
        self.seed = seed

    def __len__(self) -> int:
        return self.length

    def __getitem__(self, i: int):
        x, y = synthetic_batch(torch.tensor([i]), self.shape, self.num_classes, self.seed)
        return x[0], int(y[0])


class DeviceBatchLoader:
    """Yields ``(images NCHW, labels)`` on ``device`` for the sampler's indices, batch by batch.

    Equivalent of ``DataLoader(dataset, batch_size, sampler)`` (task.py:263) with the dataset
    generated in place on the GPU.  ``drop_last`` defaults to False like DataLoader.
    """

    def __init__(self, dataset: SyntheticImageDataset, batch_size: int, sampler=None,
                 device: torch.device = torch.device("cpu"), drop_last: bool = False,
                 dtype: torch.dtype = torch.float32, cache_batches: int = 0):
        self.ds = dataset
        self.batch_size = batch_size
        self.sampler = sampler
        self.device = device
        self.drop_last = drop_last
        self.dtype = dtype
        self.cache_batches = cache_batches
        self._cache: List[Tuple[torch.Tensor, torch.Tensor]] = []

    def _indices(self) -> List[int]:
        return list(iter(self.sampler)) if self.sampler is not None else list(range(len(self.ds)))

    def __len__(self) -> int:
        n = len(self.sampler) if self.sampler is not None else len(self.ds)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        idx = self._indices()
        for b, s in enumerate(range(0, len(idx), self.batch_size)):
            chunk = idx[s:s + self.batch_size]
            if self.drop_last and len(chunk) < self.batch_size:
                break
            if self.cache_batches and b < len(self._cache):
                yield self._cache[b]
                continue
            t = torch.tensor(chunk, dtype=torch.int64, device=self.device)
            x, y = synthetic_batch(t, self.ds.shape, self.ds.num_classes, self.ds.seed, self.dtype)
            if self.cache_batches and len(self._cache) < self.cache_batches:
                self._cache.append((x, y))
            yield x, y
