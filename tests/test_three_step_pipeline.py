"""BASELINE config 5 pipeline (preprocess -> train -> eval -> gated deploy) end to end on CPU:
compiled to kfp-v2 IR, executed by the local orchestrator, training through the launcher and
task.py on native-loader records."""
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "examples"))


def _run(tmp_path, baseline):
    import three_step_pipeline as P
    serving = tmp_path / f"serving_{int(baseline)}"
    rc = P.main(["--gpus", "0", "--arch", "mnist_cnn", "--dataset", "mnist", "--epochs", "2",
                 "--batch-size", "64", "--n-train", "512", "--n-test", "128", "--lr", "0.05",
                 "--baseline-accuracy", str(baseline), "--serving-dir", str(serving),
                 "--spec", str(tmp_path / "spec.json")])
    return rc, serving


def test_three_step_pipeline_deploys_when_above_baseline(tmp_path, gcs_root):
    rc, serving = _run(tmp_path, 0.0)
    assert rc == 0
    spec = json.load(open(tmp_path / "spec.json"))
    dag = spec["pipelineSpec"]["root"]["dag"]["tasks"]
    assert {"preprocess", "train", "evaluate"} <= set(dag)
    assert any(os.path.basename(root) for root, _, files in os.walk(serving) if "model.pth" in files)


def test_three_step_pipeline_gate_blocks_deploy(tmp_path, gcs_root):
    rc, serving = _run(tmp_path, 101.0)
    assert rc == 0  # a skipped deploy is a successful run
    assert not serving.exists()
