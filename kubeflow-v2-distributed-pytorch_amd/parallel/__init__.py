"""Data parallelism over RCCL (``torch.distributed`` backend "nccl" is RCCL on ROCm).

* :class:`DistributedDataParallel` — one process per MI355X, flat in-place gradient buckets
  all-reduced during backward (replaces torch DDP at task.py:189/194);
* :class:`DataParallel` — single-process multi-GPU replicate/scatter/gather (the reference's
  path (d), task.py:201-208);
* :class:`DistributedSampler` — disjoint per-rank index shards (task.py:260), with
  ``set_epoch`` honoured (SURVEY §5.9 quirk fixed);
* :mod:`.dist_utils` — rank/world helpers and the task.py rendezvous math.
"""
from .ddp import DistributedDataParallel, CollectiveSequenceError  # noqa: F401
from .data_parallel import DataParallel  # noqa: F401
from .sampler import DistributedSampler  # noqa: F401
from . import dist_utils  # noqa: F401
