"""Small pipelines used by the orchestrator tests (components need a source file)."""
from typing import NamedTuple

from mipipe.dsl import (component, pipeline, Condition, InputPath, OutputPath, Input, Output,
                        Dataset, Metrics, Model, importer, Artifact)


@component
def make_data(n: int, out_path: OutputPath(Dataset)) -> int:
    with open(out_path, "w") as f:
        for i in range(n):
            f.write(f"{i}\n")
    return n * 2


@component
def consume(data_path: InputPath(Dataset), scale: float, metrics: Output[Metrics]) -> NamedTuple(
        "Out", [("total", float), ("note", str)]):
    from collections import namedtuple
    vals = [int(x) for x in open(data_path).read().split()]
    total = sum(vals) * scale
    metrics.log_metric("total", total)
    return namedtuple("Out", ["total", "note"])(total, "ok")


@component
def gate_step(x: float) -> str:
    return f"passed {x}"


@component
def flaky(marker_path: str) -> str:
    import os
    if not os.path.exists(marker_path):
        open(marker_path, "w").write("1")
        raise SystemExit(3)
    return "recovered"


@component
def boom() -> str:
    raise RuntimeError("boom")


@component
def after_boom() -> str:
    return "should not run"


@pipeline(name="unit-pipe")
def unit_pipe(n: int = 4, scale: float = 1.5, threshold: float = 5.0):
    d = make_data(n)
    c = consume(d.outputs["out"], scale)
    with Condition(c.outputs["total"] >= threshold):
        gate_step(c.outputs["total"])


@pipeline(name="retry-pipe")
def retry_pipe(marker: str):
    flaky(marker).set_retry(2).set_caching_options(False)


@pipeline(name="fail-pipe")
def fail_pipe():
    b = boom()
    after_boom().after(b)


@component
def read_imported(a: Input[Artifact]) -> str:
    return open(a.path).read()


@pipeline(name="import-pipe")
def import_pipe(uri: str = "gs://bkt/hello.txt"):
    imp = importer(artifact_uri=uri, artifact_class=Artifact)
    read_imported(imp.output)
