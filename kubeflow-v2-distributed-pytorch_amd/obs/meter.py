"""Throughput meter with warmup exclusion and device-synchronised timing.

The reference has no throughput metric at all (second-resolution timestamps
only).  ``ThroughputMeter`` records a HIP event per step and synchronises only when a rate
is requested, so it adds no host sync to the hot loop.
"""
from __future__ import annotations

import time
from typing import List, Optional

import torch

__all__ = ["ThroughputMeter"]


class ThroughputMeter:
    def __init__(self, device: torch.device, warmup_steps: int = 2):
        self.device = device
        self.warmup = warmup_steps
        self.steps = 0
        self.samples = 0
        self._t0: Optional[float] = None
        self._ev0 = None
        self._last_end = None
        self._cuda = device.type == "cuda"

    def step_begin(self) -> None:
        if self.steps == self.warmup and self._t0 is None:
            if self._cuda:
                self._ev0 = torch.cuda.Event(enable_timing=True)
                self._ev0.record()
            self._t0 = time.perf_counter()

    def step_end(self, batch: int) -> None:
        if self._t0 is not None:
            self.samples += batch
            if self._cuda:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
                self._last_end = ev
        self.steps += 1

    def elapsed(self) -> float:
        if self._t0 is None:
            return 0.0
        if self._cuda and self._ev0 is not None and self._last_end is not None:
            self._last_end.synchronize()
            return self._ev0.elapsed_time(self._last_end) / 1e3
        return time.perf_counter() - self._t0

    def samples_per_sec(self) -> float:
        e = self.elapsed()
        return self.samples / e if e > 0 else 0.0
