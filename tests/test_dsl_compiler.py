"""DSL -> kfp v2 IR: the reference pipeline's exact structure (nb:218-221), naming and typing
rules, conditions, importers, NamedTuple outputs."""
import json
import os

import pytest

from mipipe.compiler import Compiler, compile_pipeline
from mipipe.dsl.component import io_name_for_path_arg, sanitize_name


def test_naming_rules():
    assert sanitize_name("download_file") == "download-file"
    assert io_name_for_path_arg("output_file_path") == "output_file"
    assert io_name_for_path_arg("input_file_path") == "input_file"
    assert io_name_for_path_arg("model_file") == "model"
    assert io_name_for_path_arg("data") == "data"


def test_reference_pipeline_ir(tmp_path):
    from examples.reference_pipeline import pipeline, download_file, train
    path = tmp_path / "dag.json"
    Compiler().compile(pipeline_func=pipeline, package_path=str(path))
    spec = json.loads(path.read_text())
    ps = spec["pipelineSpec"]
    assert ps["schemaVersion"] == "2.0.0"
    assert ps["pipelineInfo"]["name"] == "download-file-local"
    tasks = ps["root"]["dag"]["tasks"]
    assert set(tasks) == {"download-file", "train"}
    dl = tasks["download-file"]
    assert dl["componentRef"]["name"] == "comp-download-file"
    assert dl["inputs"]["parameters"]["bucket_name"] == {
        "runtimeValue": {"constantValue": {"stringValue": "test-pkl"}}}
    assert dl["inputs"]["parameters"]["source_blob_name"]["runtimeValue"]["constantValue"] == {
        "stringValue": "task.py"}
    tr = tasks["train"]
    assert tr["dependentTasks"] == ["download-file"]
    assert tr["inputs"]["artifacts"]["input_file"] == {
        "taskOutputArtifact": {"outputArtifactKey": "output_file", "producerTask": "download-file"}}
    assert tr["inputs"]["parameters"]["replica_count"] == {"componentInputParameter": "replica_count"}
    comps = ps["components"]
    assert comps["comp-download-file"]["outputDefinitions"]["artifacts"]["output_file"] == {
        "artifactType": {"schemaTitle": "system.Artifact", "schemaVersion": "0.0.1"}}
    assert comps["comp-download-file"]["inputDefinitions"]["parameters"] == {
        "bucket_name": {"type": "STRING"}, "source_blob_name": {"type": "STRING"}}
    assert comps["comp-train"]["inputDefinitions"]["parameters"]["replica_count"] == {"type": "INT"}
    assert comps["comp-train"]["outputDefinitions"]["parameters"]["Output"] == {"type": "DOUBLE"}
    assert comps["comp-train"]["outputDefinitions"]["artifacts"]["metrics"]["artifactType"][
        "schemaTitle"] == "system.Metrics"
    # float pipeline param -> DOUBLE; default lands in runtimeConfig
    assert ps["root"]["inputDefinitions"]["parameters"]["baseline_accuracy"] == {"type": "DOUBLE"}
    assert spec["runtimeConfig"]["parameters"]["baseline_accuracy"] == {"doubleValue": 70.0}
    ex = ps["deploymentSpec"]["executors"]["exec-download-file"]["container"]
    assert ex["args"] == ["--executor_input", "{{$}}", "--function_to_execute", "download_file"]
    assert "def download_file(" in ex["command"][-1]
    assert "google-cloud-storage" in ex["command"][2]
    assert ex["image"] == "python:3.7"


def test_condition_compiles_to_subdag():
    from tests.fixtures.pipes import unit_pipe
    spec = compile_pipeline(unit_pipe)
    root = spec["pipelineSpec"]["root"]["dag"]["tasks"]
    assert set(root) == {"make-data", "consume", "condition-1"}
    cond = root["condition-1"]
    assert cond["dependentTasks"] == ["consume"]
    assert cond["triggerPolicy"]["condition"] == (
        "inputs.parameters['pipelineparam--consume-total'].double_value >= "
        "inputs.parameters['pipelineparam--threshold'].double_value")
    sub = spec["pipelineSpec"]["components"]["comp-condition-1"]
    assert "gate-step" in sub["dag"]["tasks"]
    assert sub["dag"]["tasks"]["gate-step"]["inputs"]["parameters"]["x"] == {
        "componentInputParameter": "pipelineparam--consume-total"}
    assert root["consume"]["inputs"]["artifacts"]["data"]["taskOutputArtifact"][
        "outputArtifactKey"] == "out"
    comp = spec["pipelineSpec"]["components"]["comp-consume"]
    assert comp["outputDefinitions"]["parameters"] == {"total": {"type": "DOUBLE"},
                                                       "note": {"type": "STRING"}}


def test_parameter_overrides_and_unknown():
    from tests.fixtures.pipes import unit_pipe
    spec = compile_pipeline(unit_pipe, pipeline_parameters={"n": 7})
    assert spec["runtimeConfig"]["parameters"]["n"] == {"intValue": "7"}
    with pytest.raises(ValueError):
        compile_pipeline(unit_pipe, pipeline_parameters={"nope": 1})


def test_component_outside_pipeline_raises():
    from tests.fixtures.pipes import make_data
    with pytest.raises(RuntimeError):
        make_data(3)
    assert make_data.python_func.__name__ == "make_data"


def test_importer_ir():
    from tests.fixtures.pipes import import_pipe
    spec = compile_pipeline(import_pipe)
    ex = spec["pipelineSpec"]["deploymentSpec"]["executors"]
    imp = [v for v in ex.values() if "importer" in v][0]["importer"]
    assert imp["typeSchema"]["schemaTitle"] == "system.Artifact"
