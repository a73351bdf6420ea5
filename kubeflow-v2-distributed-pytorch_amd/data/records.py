"""Binary image-record datasets + the native multi-threaded loader.

Record layout = CIFAR-10 binary (``[label byte][C planes of H*W uint8]``, 3073 bytes for
32x32x3), the format ``torchvision.datasets.CIFAR10`` downloads and task.py decodes
(task.py:246-263).  There is no network here, so the pipeline's *preprocess* step writes such
files from a deterministic, learnable generator (:func:`write_synthetic_dataset`); the *train*
and *eval* steps read them through :class:`RecordDataLoader`, which drives the C++
``RecordLoader`` (csrc/runtime/loader.cpp: memory-mapped files, worker threads, RandomCrop
(padding) + RandomHorizontalFlip + Normalize, ordered prefetch ring) and hands each batch to the
GPU through a pinned staging buffer and one non-blocking copy.

:func:`reference_transform` is the plain-NumPy definition of the per-sample transform the
native loader implements (tests compare the two bit-for-bit).
"""
from __future__ import annotations

import os
from typing import Iterator, List, Optional, Sequence, Tuple

import numpy as np
import torch

from mipipe.parallel.sampler import DistributedSampler

__all__ = ["write_records", "read_records", "write_synthetic_dataset", "reference_transform",
           "RecordDataLoader", "CIFAR10_MEAN", "CIFAR10_STD", "dataset_files"]

# task.py:249-251
CIFAR10_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR10_STD = (0.2023, 0.1994, 0.2010)
MNIST_MEAN = (0.1307,)
MNIST_STD = (0.3081,)

_MASK64 = (1 << 64) - 1


def write_records(path: str, images: np.ndarray, labels: np.ndarray) -> None:
    """images uint8 [N, C, H, W], labels [N] (< 256) -> CIFAR-binary record file."""
    images = np.ascontiguousarray(images, dtype=np.uint8)
    n = images.shape[0]
    rec = np.empty((n, 1 + images[0].size), dtype=np.uint8)
    rec[:, 0] = np.asarray(labels, dtype=np.uint8)
    rec[:, 1:] = images.reshape(n, -1)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    rec.tofile(path)


def read_records(path: str, shape: Sequence[int]) -> Tuple[np.ndarray, np.ndarray]:
    C, H, W = shape
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 1 + C * H * W)
    return raw[:, 1:].reshape(-1, C, H, W), raw[:, 0].astype(np.int64)


def write_synthetic_dataset(out_dir: str, name: str = "cifar10", n_train: int = 10000,
                            n_test: int = 2000, seed: int = 0, num_classes: int = 10) -> dict:
    """Learnable synthetic dataset in CIFAR-binary layout: class template (low-frequency
    pattern) + per-sample noise, quantised to uint8.  Returns a manifest dict."""
    shape = {"cifar10": (3, 32, 32), "mnist": (1, 28, 28)}[name]
    C, H, W = shape
    rng = np.random.default_rng(seed)
    base = rng.normal(0.0, 1.0, size=(num_classes, C, H // 4, W // 4))
    templates = np.kron(base, np.ones((1, 1, 4, 4)))[:, :, :H, :W]

    def make(n, split_seed):
        r = np.random.default_rng(seed * 1000 + split_seed)
        y = r.integers(0, num_classes, size=n)
        x = 0.8 * templates[y] + r.normal(0.0, 1.0, size=(n, C, H, W))
        img = np.clip(x * 40.0 + 128.0, 0, 255).astype(np.uint8)
        return img, y

    files = {}
    os.makedirs(out_dir, exist_ok=True)
    for split, n, s in (("train", n_train, 1), ("test", n_test, 2)):
        img, y = make(n, s)
        path = os.path.join(out_dir, f"{name}_{split}.bin")
        write_records(path, img, y)
        files[split] = path
    return {"name": name, "shape": list(shape), "num_classes": num_classes,
            "n_train": n_train, "n_test": n_test, "files": files}


def dataset_files(data_dir: str, name: str, split: str) -> List[str]:
    """Record files of ``split`` in ``data_dir``: our ``<name>_<split>.bin`` or the original
    CIFAR-10 binary names (data_batch_*.bin / test_batch.bin)."""
    own = os.path.join(data_dir, f"{name}_{split}.bin")
    if os.path.exists(own):
        return [own]
    if name == "cifar10":
        d = os.path.join(data_dir, "cifar-10-batches-bin")
        d = d if os.path.isdir(d) else data_dir
        names = ([f"data_batch_{i}.bin" for i in range(1, 6)] if split == "train"
                 else ["test_batch.bin"])
        found = [os.path.join(d, n) for n in names if os.path.exists(os.path.join(d, n))]
        if found:
            return found
    return []


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _MASK64
    return x ^ (x >> 31)


def reference_transform(img: np.ndarray, index: int, epoch: int, seed: int, train: bool,
                        pad: int, flip: bool, mean, std) -> np.ndarray:
    """NumPy definition of loader.cpp's per-sample transform (uint8 CHW -> float32 CHW)."""
    C, H, W = img.shape
    dy = dx = 0
    fl = False
    if train:
        h = _splitmix64(seed ^ _splitmix64(((epoch * 0x100000001B3) & _MASK64) ^ index))
        if pad > 0:
            dy = int(h % (2 * pad + 1)) - pad
            dx = int((h >> 16) % (2 * pad + 1)) - pad
        fl = flip and bool((h >> 40) & 1)
    padded = np.zeros((C, H + 2 * pad, W + 2 * pad), dtype=np.float32)
    padded[:, pad:pad + H, pad:pad + W] = img
    out = padded[:, pad + dy:pad + dy + H, pad + dx:pad + dx + W]
    if fl:
        out = out[:, :, ::-1]
    m = np.asarray(mean, np.float32)[:, None, None]
    s = np.asarray(std, np.float32)[:, None, None]
    return (out * (1.0 / (255.0 * s)) + (-m / s)).astype(np.float32)


class RecordDataLoader:
    """Iterates (x [B,C,H,W] float32, y [B] int64) batches of this rank's shard.

    ``sampler`` follows :class:`DistributedSampler` semantics (``set_epoch`` reshuffles);
    batches land on ``device`` (pinned staging + non_blocking copy for GPU devices)."""

    def __init__(self, files: Sequence[str], shape: Sequence[int], batch_size: int,
                 sampler: Optional[DistributedSampler] = None, train: bool = True,
                 pad: int = 4, flip: bool = True, mean=CIFAR10_MEAN, std=CIFAR10_STD,
                 seed: int = 0, workers: int = 8, prefetch: int = 4, drop_last: bool = False,
                 device: Optional[torch.device] = None):
        from mipipe.runtime import runtime, runtime_available
        self.shape = tuple(shape)
        self.batch_size = batch_size
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.train, self.pad, self.flip = train, pad, flip
        self.mean, self.std, self.seed = tuple(mean), tuple(std), seed
        self.epoch = 0
        self.files = list(files)
        self.native = runtime_available()
        if self.native:
            cfg = runtime().LoaderConfig()
            cfg.files = self.files
            cfg.C, cfg.H, cfg.W = self.shape
            cfg.batch = batch_size
            cfg.train, cfg.pad, cfg.flip = train, pad if train else 0, flip and train
            cfg.mean, cfg.std = list(map(float, mean)), list(map(float, std))
            cfg.seed, cfg.workers, cfg.prefetch, cfg.drop_last = seed, workers, prefetch, drop_last
            self._ld = runtime().RecordLoader(cfg)
            n = len(self._ld)
        else:
            self._imgs, self._labels = [], []
            for f in self.files:
                x, y = read_records(f, self.shape)
                self._imgs.append(x)
                self._labels.append(y)
            self._imgs = np.concatenate(self._imgs) if self._imgs else np.zeros((0, *self.shape), np.uint8)
            self._labels = np.concatenate(self._labels) if self._labels else np.zeros(0, np.int64)
            n = len(self._labels)
        self.num_samples_total = n
        self.sampler = sampler if sampler is not None else DistributedSampler(n, shuffle=train,
                                                                               seed=seed)
        self.drop_last = drop_last
        pin = self.device.type == "cuda"
        C, H, W = self.shape
        self._stage = [(torch.empty(batch_size, C, H, W, dtype=torch.float32, pin_memory=pin),
                        torch.empty(batch_size, dtype=torch.int64, pin_memory=pin))
                       for _ in range(2)]

    def __len__(self) -> int:
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else -(-n // self.batch_size)

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
        self.sampler.set_epoch(epoch)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        self.epoch = getattr(self.sampler, "epoch", self.epoch)  # follow sampler.set_epoch
        idx = list(iter(self.sampler))
        if self.native:
            self._ld.start_epoch(idx, self.epoch)
            k = 0
            events = [None, None]
            while True:
                xs, ys = self._stage[k % 2]
                if events[k % 2] is not None:
                    events[k % 2].synchronize()  # the H2D copy out of this staging buffer is done
                n = self._ld.next_into(xs.data_ptr(), ys.data_ptr())
                if n == 0:
                    return
                out = self._to_device(xs[:n], ys[:n])
                if self.device.type == "cuda":
                    ev = torch.cuda.Event()
                    ev.record(torch.cuda.current_stream(self.device))
                    events[k % 2] = ev
                yield out
                k += 1
        else:
            for b in range(len(self)):
                sl = idx[b * self.batch_size:(b + 1) * self.batch_size]
                x = np.stack([reference_transform(self._imgs[i], i, self.epoch, self.seed,
                                                  self.train, self.pad if self.train else 0,
                                                  self.flip and self.train, self.mean, self.std)
                              for i in sl])
                yield self._to_device(torch.from_numpy(x), torch.from_numpy(self._labels[sl]))

    def _to_device(self, x: torch.Tensor, y: torch.Tensor):
        if self.device.type == "cpu":
            return x.clone(), y.clone()
        return x.to(self.device, non_blocking=True), y.to(self.device, non_blocking=True)
