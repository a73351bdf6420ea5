"""Per-rank dataset sharding (task.py:260 ``DistributedSampler(dataset=train_set)``).

Pure index arithmetic — no collective: rank r takes indices
r, r+W, r+2W, ... of a (optionally epoch-seeded) permutation padded to a multiple of W.
Unlike the reference, the trainer calls ``set_epoch`` every epoch.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch

__all__ = ["DistributedSampler"]


class DistributedSampler(torch.utils.data.Sampler):
    def __init__(self, dataset_or_len, num_replicas: Optional[int] = None,
                 rank: Optional[int] = None, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        import torch.distributed as dist
        n = dataset_or_len if isinstance(dataset_or_len, int) else len(dataset_or_len)
        if num_replicas is None:
            num_replicas = dist.get_world_size() if dist.is_initialized() else 1
        if rank is None:
            rank = dist.get_rank() if dist.is_initialized() else 0
        if not 0 <= rank < num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.n, self.num_replicas, self.rank = n, num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and n % num_replicas:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def __iter__(self) -> Iterator[int]:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(self.n, generator=g).tolist()
        else:
            indices = list(range(self.n))
        if not self.drop_last:
            pad = self.total_size - len(indices)
            if pad > 0:
                indices += (indices * math.ceil(pad / max(len(indices), 1)))[:pad]
        else:
            indices = indices[:self.total_size]
        return iter(indices[self.rank:self.total_size:self.num_replicas])

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
