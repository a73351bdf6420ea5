"""Structured per-rank JSON-lines logs: one ``rank<k>.jsonl`` per rank under
``$MIPIPE_LOG_DIR`` (or a given directory), each line ``{"ts", "rank", "event", ...}``; rank 0
can merge them into one job-level summary with :func:`aggregate`."""
from __future__ import annotations

import glob
import json
import os
import time
from typing import Any, Dict, List, Optional


class JsonlLogger:
    def __init__(self, rank: int, log_dir: Optional[str] = None):
        self.rank = rank
        d = log_dir or os.environ.get("MIPIPE_LOG_DIR", "")
        self.path = None
        self._f = None
        if d:
            os.makedirs(d, exist_ok=True)
            self.path = os.path.join(d, f"rank{rank}.jsonl")
            self._f = open(self.path, "a", buffering=1)

    def log(self, event: str, **fields: Any) -> None:
        if self._f is None:
            return
        rec = {"ts": time.time(), "rank": self.rank, "event": event}
        rec.update(fields)
        self._f.write(json.dumps(rec, default=str) + "\n")

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None


def read_all(log_dir: str) -> List[Dict[str, Any]]:
    out = []
    for p in sorted(glob.glob(os.path.join(log_dir, "rank*.jsonl"))):
        with open(p) as f:
            out.extend(json.loads(line) for line in f if line.strip())
    return out


def aggregate(log_dir: str, event: str = "step") -> Dict[str, Any]:
    """Job-level summary of per-rank ``step`` records: total samples/s (sum over ranks of each
    rank's mean throughput), slowest rank, step count."""
    recs = [r for r in read_all(log_dir) if r.get("event") == event]
    by_rank: Dict[int, List[Dict[str, Any]]] = {}
    for r in recs:
        by_rank.setdefault(int(r["rank"]), []).append(r)
    per_rank = {k: sum(float(x.get("samples_per_sec", 0.0)) for x in v) / max(1, len(v))
                for k, v in by_rank.items()}
    return {"ranks": len(by_rank), "steps": max((len(v) for v in by_rank.values()), default=0),
            "samples_per_sec_job": sum(per_rank.values()),
            "slowest_rank": min(per_rank, key=per_rank.get) if per_rank else None,
            "per_rank": per_rank}
