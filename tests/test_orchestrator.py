"""Local orchestrator: artifact passing, parameter outputs, conditions, caching, retries,
fail-fast, importer, client API."""
import json
import os

import pytest

from mipipe.client import AIPlatformClient
from mipipe.compiler import Compiler
from mipipe.orchestrator import PipelineRunner
from mipipe.orchestrator import cel


def _compile(p, tmp_path, name="p.json"):
    path = tmp_path / name
    Compiler().compile(p, str(path))
    return str(path)


def test_cel_subset():
    params = {"a": {"doubleValue": 3.5}, "b": {"intValue": "2"}, "s": {"stringValue": "x"}}
    assert cel.evaluate("inputs.parameters['a'].double_value >= 3.0", params)
    assert not cel.evaluate("inputs.parameters['b'].int_value > 2", params)
    assert cel.evaluate("inputs.parameters['s'].string_value == 'x' && !(1 > 2)", params)
    with pytest.raises(ValueError):
        cel.evaluate("__import__('os')", params)


def test_run_with_condition_true_and_false(gcs_root, tmp_path):
    from tests.fixtures.pipes import unit_pipe
    spec = json.load(open(_compile(unit_pipe, tmp_path)))
    r = PipelineRunner(spec, pipeline_root="gs://b/root", echo_logs=False).run()
    assert r["state"] == "PIPELINE_STATE_SUCCEEDED", r["tasks"]
    t = r["tasks"]
    assert t["make-data"]["outputs"]["parameters"]["Output"] == {"intValue": "8"}
    assert t["consume"]["outputs"]["parameters"]["total"] == {"doubleValue": 9.0}  # (0+1+2+3)*1.5
    assert t["consume"]["outputs"]["artifacts"]["metrics"][0]["metadata"]["total"] == 9.0
    assert t["condition-1/gate-step"]["state"] == "SUCCEEDED"
    assert t["condition-1/gate-step"]["outputs"]["parameters"]["Output"]["stringValue"] == "passed 9.0"
    data_uri = t["make-data"]["outputs"]["artifacts"]["out"][0]["uri"]
    assert data_uri.startswith("gs://b/root/")
    r2 = PipelineRunner(spec, pipeline_root="gs://b/root", parameter_values={"threshold": 100.0},
                        echo_logs=False, run_id="second").run()
    assert r2["tasks"]["condition-1"]["state"] == "SKIPPED"
    # caching: identical inputs reuse the first run's outputs
    assert r2["tasks"]["make-data"]["state"] == "CACHED"


def test_retry_and_fail_fast(gcs_root, tmp_path):
    from tests.fixtures.pipes import retry_pipe, fail_pipe
    marker = str(tmp_path / "marker")
    spec = json.load(open(_compile(retry_pipe, tmp_path, "r.json")))
    r = PipelineRunner(spec, parameter_values={"marker": marker}, echo_logs=False).run()
    assert r["state"] == "PIPELINE_STATE_SUCCEEDED"
    assert r["tasks"]["flaky"]["attempts"] == 2
    spec = json.load(open(_compile(fail_pipe, tmp_path, "f.json")))
    r = PipelineRunner(spec, echo_logs=False).run()
    assert r["state"] == "PIPELINE_STATE_FAILED"
    assert r["tasks"]["boom"]["state"] == "FAILED"
    assert r["tasks"]["after-boom"]["state"] == "CANCELLED"


def test_importer_and_client(gcs_root, tmp_path):
    from mipipe.storage import gcs
    from tests.fixtures.pipes import import_pipe
    gcs.Client().bucket("bkt").blob("hello.txt").upload_from_string("hi there")
    path = _compile(import_pipe, tmp_path, "i.json")
    client = AIPlatformClient("proj", "region", echo_logs=False)
    resp = client.create_run_from_job_spec(path, pipeline_root="gs://bkt/pr")
    assert resp["name"].startswith("projects/proj/locations/region/pipelineJobs/")
    res = client.wait_for_run(resp["runId"])
    assert res["state"] == "PIPELINE_STATE_SUCCEEDED"
    run = client.get_run(resp["runId"])
    assert run["tasks"]["read-imported"]["outputs"]["parameters"]["Output"]["stringValue"] == "hi there"
