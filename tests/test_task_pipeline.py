"""task.py flag parity + rank math, CPU training/resume/export, sampler, synthetic data, and
the reference pipeline end-to-end on the local orchestrator (BASELINE config 1: CPU/gloo,
world_size=1, local kfp run)."""
import json
import os
import sys

import pytest
import torch

from mipipe.train import task as T

# task.py:56-94 — (dest, default) of every reference flag
REFERENCE_FLAGS = {
    "local_rank": None, "num_epochs": 100, "batch_size": 1024, "learning_rate": 0.1,
    "random_seed": 0, "model_filename": "resnet_distributed.pth", "arch": "resnet18",
    "momentum": 0.9, "weight_decay": 1e-4, "pretrained": False, "local_training": False,
    "rank": -1, "multiprocessing_distributed": False, "gpu": None, "workers": 4,
    "dist_backend": "nccl",
}


def test_flag_parity(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("AIP_MODEL_DIR", raising=False)
    a = T.build_parser().parse_args([])
    for k, v in REFERENCE_FLAGS.items():
        assert getattr(a, k) == v, k
    assert a.world_size == -1 and a.model_dir == ""
    # reference spellings parse
    a = T.build_parser().parse_args(["--dist-url=env://", "--multiprocessing-distributed",
                                     "--num_epochs=2", "-a", "resnet50", "--wd", "5e-4",
                                     "--world-size", "3", "--dist-backend", "gloo"])
    assert a.multiprocessing_distributed and a.num_epochs == 2 and a.arch == "resnet50"
    assert a.weight_decay == 5e-4 and a.world_size == 3 and a.dist_url == "env://"
    monkeypatch.setenv("AIP_MODEL_DIR", "gs://b/model/")
    assert T.build_parser().parse_args([]).model_dir == "gs://b/model/"


def test_rank_math():
    from mipipe.parallel import dist_utils as D
    assert D.global_world_size(3, 2) == 6        # task.py:120
    assert [D.global_rank(n, 2, g) for n in range(3) for g in range(2)] == list(range(6))  # :146


def test_sampler_shards():
    from mipipe.parallel import DistributedSampler
    n, W = 10, 3
    shards = [list(DistributedSampler(n, W, r, seed=1)) for r in range(W)]
    assert all(len(s) == 4 for s in shards)
    assert set(sum(shards, [])) == set(range(n))
    s = DistributedSampler(n, W, 0, seed=1)
    e0 = list(s)
    s.set_epoch(1)
    assert list(s) != e0


def test_synthetic_deterministic_and_learnable():
    from mipipe.data.synthetic import SyntheticImageDataset, synthetic_batch
    idx = torch.arange(5)
    x1, y1 = synthetic_batch(idx, (1, 8, 8), 10, 3)
    x2, y2 = synthetic_batch(idx, (1, 8, 8), 10, 3)
    assert torch.equal(x1, x2) and torch.equal(y1, y2)
    ds = SyntheticImageDataset("mnist", 100)
    img, lab = ds[7]
    assert img.shape == (1, 28, 28) and 0 <= lab < 10
    # same-class images correlate (template), different classes do not
    xs, ys = synthetic_batch(torch.arange(200), (1, 8, 8), 4, 0)
    a = xs[ys == 0][:2].reshape(2, -1)
    assert torch.nn.functional.cosine_similarity(a[0:1], a[1:2]).item() > 0.1


def test_train_resume_export(tmp_path, monkeypatch):
    monkeypatch.setenv("MIPIPE_FORCE_CPU", "1")
    monkeypatch.delenv("AIP_MODEL_DIR", raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    out = tmp_path / "out"
    args = ["--arch", "mnist_cnn", "--dataset", "mnist", "--batch_size", "32",
            "--train-samples", "128", "--test-samples", "64", "--local_training",
            "--model_dir", str(out), "--learning_rate", "0.05", "--log-every", "0",
            "--metrics-file", str(tmp_path / "m.json")]
    assert T.main(args + ["--num_epochs", "1"]) == 0
    m = json.loads((tmp_path / "m.json").read_text())
    assert m["steps"] == 4 and m["world_size"] == 1
    sd = torch.load(out / "resnet_distributed.pth", weights_only=True)
    assert "conv1.weight" in sd
    ck = torch.load(out / "checkpoint.pth.tar", weights_only=True)
    assert ck["epoch"] == 1 and set(ck) >= {"epoch", "arch", "best_acc1", "state_dict", "optimizer"}
    assert T.main(args + ["--num_epochs", "2", "--resume"]) == 0
    m = json.loads((tmp_path / "m.json").read_text())
    assert m["steps"] == 4  # resumed at epoch 1: only epoch 1 ran
    assert torch.load(out / "checkpoint.pth.tar", weights_only=True)["epoch"] == 2


def test_fault_injection_fail_fast(tmp_path):
    from mipipe.launch import LaunchSpec, launch
    env = {"MIPIPE_FAULT_INJECT": "1:1:9", "MIPIPE_FORCE_CPU": "1",
           "PYTHONPATH": os.path.dirname(os.path.dirname(os.path.abspath(__file__)))}
    task = os.path.join(env["PYTHONPATH"], "kubeflow-v2-distributed-pytorch_amd", "train", "task.py")
    rc = launch(LaunchSpec(command=[sys.executable, task, "--arch", "mnist_cnn", "--dataset",
                                    "mnist", "--batch_size", "16", "--train-samples", "256",
                                    "--test-samples", "32", "--num_epochs", "3",
                                    "--log-every", "0", "--local_training", "--model_dir",
                                    str(tmp_path), "--dist-timeout", "60"],
                           replica_count=2, env=env, echo=False, grace_period=5.0,
                           timeout=240))
    assert rc == 9


def test_reference_pipeline_end_to_end(gcs_root, tmp_path, monkeypatch):
    monkeypatch.setenv("MIPIPE_FORCE_CPU", "1")
    monkeypatch.chdir(tmp_path)
    from examples import reference_pipeline as rp
    rc = rp.main(["--replicas", "1", "--gpus-per-replica", "0", "--epochs", "1",
                  "--spec", str(tmp_path / "dag.json")])
    assert rc == 0
    runs = list((gcs_root / "test-pkl" / "pipeline_root").iterdir())
    run = json.loads((runs[0] / "run.json").read_text())
    assert run["state"] == "PIPELINE_STATE_SUCCEEDED"
    assert run["runtimeParameters"]["baseline_accuracy"] == {"doubleValue": 80.0}
    tr = run["tasks"]["train"]["outputs"]
    assert tr["parameters"]["Output"]["doubleValue"] >= 0.0
    assert tr["artifacts"]["metrics"][0]["metadata"]["steps"] > 0
    models = list((gcs_root / "test-pkl" / "jobs").glob("*/model/resnet_distributed.pth"))
    assert models, "model not exported to AIP_MODEL_DIR"
    sd = torch.load(models[0], weights_only=True)
    assert any(k.startswith("module.") for k in sd)  # DDP-wrapped, like the reference


def test_find_pretrained_prefers_imagenet1k_v1(tmp_path, monkeypatch):
    """With several torchvision weight versions cached, pretrained=True means IMAGENET1K_V1
    (torchvision 0.8, the reference's container nb:137), independent of hash sort order."""
    from mipipe.models import find_pretrained
    ck = tmp_path / "hub" / "checkpoints"
    ck.mkdir(parents=True)
    for f in ("resnet50-11ad3fa6.pth", "resnet50-0676ba61.pth"):  # V2 sorts first
        (ck / f).write_bytes(b"")
    (ck / "inception_v3_google-0cc3c7bd.pth").write_bytes(b"")
    monkeypatch.setenv("TORCH_HOME", str(tmp_path))
    assert find_pretrained("resnet50") == str(ck / "resnet50-0676ba61.pth")
    assert find_pretrained("inception_v3") == str(ck / "inception_v3_google-0cc3c7bd.pth")
    (ck / "resnet18-aaaaaaaa.pth").write_bytes(b"")
    (ck / "resnet18-bbbbbbbb.pth").write_bytes(b"")
    with pytest.warns(UserWarning, match="IMAGENET1K_V1"):
        assert find_pretrained("resnet18") == str(ck / "resnet18-aaaaaaaa.pth")


def test_pretrained_from_local_torchvision_file(tmp_path, monkeypatch, capsys):
    """--pretrained (task.py:166-168) loads a torchvision-format state_dict from
    --pretrained-weights or the torchvision cache with a weights-only loader."""
    from mipipe.models import create_model, find_pretrained, load_pretrained
    torch.manual_seed(3)
    src = create_model("resnet18", num_classes=10)
    path = tmp_path / "hub" / "checkpoints" / "resnet18-f37072fd.pth"
    path.parent.mkdir(parents=True)
    torch.save({("module." + k): v for k, v in src.state_dict().items()}, path)
    monkeypatch.setenv("TORCH_HOME", str(tmp_path))
    assert find_pretrained("resnet18") == str(path)
    assert find_pretrained("resnet50") is None
    dst = create_model("resnet18", num_classes=10)
    load_pretrained(dst, str(path))
    for (k, a), (_, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert torch.equal(a, b), k
    # through task.py: the exported model equals the pre-trained weights after 0 steps
    monkeypatch.setenv("MIPIPE_FORCE_CPU", "1")
    monkeypatch.delenv("AIP_MODEL_DIR", raising=False)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    out = tmp_path / "out"
    rc = T.main(["--arch", "resnet18", "--num_classes", "10", "--pretrained",
                 "--pretrained-weights", str(path), "--dataset", "cifar10", "--batch_size", "8",
                 "--train-samples", "8", "--test-samples", "8", "--num_epochs", "1",
                 "--learning_rate", "0.0", "--momentum", "0", "--wd", "0", "--local_training",
                 "--model_dir", str(out), "--log-every", "0"])
    assert rc == 0
    assert "loaded pre-trained weights" in capsys.readouterr().out
    sd = torch.load(out / "resnet_distributed.pth", weights_only=True)
    assert torch.equal(sd["conv1.weight"], src.state_dict()["conv1.weight"])
