"""GPU clock / power sampling for benchmark lines.

Box-to-box spread of the headline number (README: 10.3k-11.3k img/s for the same code) was
attributed to compute-clock differences; this makes that attribution checkable.  A daemon
thread samples the amdgpu hwmon files of the device under test (sysfs reads only, no
subprocess in the timed loop): ``freq1_input`` (shader clock, Hz), ``freq2_input`` (memory
clock), ``power1_average`` / ``power1_input`` (µW), ``temp*_input`` (m°C).  The device is found by
the PCI bus id torch reports for it.  Where sysfs is not readable the sampler reports
``{"source": "unavailable"}`` and the bench line says so.
"""
from __future__ import annotations

import glob
import os
import threading
import time
from typing import Dict, List, Optional

__all__ = ["ClockSampler", "hwmon_dir_for"]


def _pci_id(dev_index: int) -> Optional[str]:
    try:
        import torch
        p = torch.cuda.get_device_properties(dev_index)
        dom = getattr(p, "pci_domain_id", 0)
        bus = getattr(p, "pci_bus_id", None)
        devid = getattr(p, "pci_device_id", 0)
        if bus is None:
            return None
        return f"{dom:04x}:{bus:02x}:{devid:02x}.0"
    except Exception:
        return None


def hwmon_dir_for(dev_index: int) -> Optional[str]:
    """hwmon directory of the GPU torch calls ``cuda:dev_index`` (None when not found)."""
    pci = _pci_id(dev_index)
    cands = []
    if pci is not None:
        cands = glob.glob(f"/sys/bus/pci/devices/{pci}/hwmon/hwmon*")
    if not cands:
        # one visible amdgpu device: take the only amdgpu hwmon that exposes a shader clock
        ams = [d for d in glob.glob("/sys/class/hwmon/hwmon*")
               if _read(os.path.join(d, "name")) == "amdgpu"
               and os.path.exists(os.path.join(d, "freq1_input"))]
        if len(ams) == 1:
            cands = ams
    return cands[0] if cands else None


def _read(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except Exception:
        return None


def _read_num(path: str) -> Optional[float]:
    v = _read(path)
    try:
        return float(v) if v is not None else None
    except ValueError:
        return None


class ClockSampler:
    """``with ClockSampler(dev) as cs: <timed loop>``; then ``cs.summary()``."""

    def __init__(self, dev_index: int = 0, period_s: float = 0.05):
        self.dir = hwmon_dir_for(dev_index)
        self.period = period_s
        self.samples: List[Dict[str, float]] = []
        self._stop = threading.Event()
        self._th: Optional[threading.Thread] = None

    def _sample(self) -> Dict[str, float]:
        d = self.dir
        out: Dict[str, float] = {}
        if d is None:
            return out
        for key, fname, scale in (("sclk_mhz", "freq1_input", 1e-6),
                                  ("mclk_mhz", "freq2_input", 1e-6),
                                  ("power_w", "power1_average", 1e-6),
                                  ("power_w", "power1_input", 1e-6)):
            if key in out:
                continue
            v = _read_num(os.path.join(d, fname))
            if v is not None:
                out[key] = v * scale
        temps = [_read_num(p) for p in sorted(glob.glob(os.path.join(d, "temp*_input")))]
        temps = [t for t in temps if t is not None]
        if temps:
            out["temp_c_max"] = max(temps) / 1e3
        return out

    def _loop(self) -> None:
        while not self._stop.is_set():
            s = self._sample()
            if s:
                self.samples.append(s)
            self._stop.wait(self.period)

    def __enter__(self) -> "ClockSampler":
        if self.dir is not None:
            self._th = threading.Thread(target=self._loop, daemon=True)
            self._th.start()
        return self

    def __exit__(self, *exc) -> None:
        self._stop.set()
        if self._th is not None:
            self._th.join(timeout=1.0)

    def summary(self) -> Dict[str, object]:
        if self.dir is None:
            return {"source": "unavailable"}
        if not self.samples:
            return {"source": self.dir, "samples": 0}
        out: Dict[str, object] = {"source": self.dir, "samples": len(self.samples)}
        keys = sorted({k for s in self.samples for k in s})
        for k in keys:
            vs = [s[k] for s in self.samples if k in s]
            out[k] = {"mean": round(sum(vs) / len(vs), 1), "min": round(min(vs), 1),
                      "max": round(max(vs), 1)}
        return out


if __name__ == "__main__":  # quick look on a GPU box
    import json
    cs = ClockSampler(0)
    with cs:
        time.sleep(0.5)
    print(json.dumps(cs.summary()))
