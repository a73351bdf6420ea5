"""Observability: roctx phase ranges (no-op when disabled), per-rank JSON-lines logs and their
aggregation, task.py --log-dir/--trace plumbing."""
import json

from mipipe.obs import trace
from mipipe.obs.log import JsonlLogger, aggregate, read_all


def test_phase_is_noop_when_disabled():
    trace.enable(False)
    with trace.phase("x"):
        pass
    assert not trace.enabled()


def test_phase_with_roctx_enabled_runs():
    trace.enable(True)  # libroctx64 ships with ROCm; ranges are harmless without a profiler
    try:
        with trace.phase("forward"):
            trace.mark("hello")
    finally:
        trace.enable(False)


def test_jsonl_logs_and_aggregate(tmp_path):
    for r, sps in ((0, 100.0), (1, 80.0)):
        lg = JsonlLogger(r, str(tmp_path))
        for s in range(3):
            lg.log("step", step=s, samples_per_sec=sps)
        lg.log("final", accuracy=0.5)
        lg.close()
    recs = read_all(str(tmp_path))
    assert len(recs) == 8 and {r["rank"] for r in recs} == {0, 1}
    agg = aggregate(str(tmp_path))
    assert agg["ranks"] == 2 and agg["steps"] == 3
    assert abs(agg["samples_per_sec_job"] - 180.0) < 1e-9 and agg["slowest_rank"] == 1
