"""The reference's exact training invocation on an MI355X.

The notebook's pipeline runs ``task.py --dist-url=env:// --multiprocessing-distributed
--num_epochs=2`` (pytorch-pipeline.ipynb nb:159-163) on every replica: that is ``mp.spawn`` of one
worker per GPU (task.py:117-124), ``init_process_group('nccl', 'env://')`` (:148-149) and
``DistributedDataParallel(model, device_ids=[gpu])`` (:189).  Here it runs on the 1-GPU box at
world size 1 (WORLD_SIZE=1 / RANK=0 as Vertex sets them for one replica), in a fresh process
(the spawning parent must not have initialised HIP), and the exported model must load into the
``module.``-prefixed torchvision layout the reference writes (task.py:282-294).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    from mipipe.launch.launcher import free_port
    e = dict(os.environ)
    for k in ("LOCAL_RANK", "GROUP_RANK"):
        e.pop(k, None)
    e.update({"WORLD_SIZE": "1", "RANK": "0", "MASTER_ADDR": "127.0.0.1",
              "MASTER_PORT": str(free_port()), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
              "PYTHONPATH": REPO + os.pathsep + e.get("PYTHONPATH", "")})
    e.update(kw)
    return e


def test_reference_invocation_mp_spawn_nccl(tmp_path):
    out = tmp_path / "model"
    args = ["--dist-url=env://", "--multiprocessing-distributed", "--num_epochs=2",
            "--local_training", "--model_dir", str(out), "--batch_size", "256",
            "--train-samples", "1024", "--test-samples", "256",
            "--metrics-file", str(tmp_path / "metrics.json")]
    r = subprocess.run([sys.executable, "-m", "mipipe.train.task"] + args, env=_env(),
                       capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    log = r.stdout + r.stderr
    (tmp_path / "log.txt").write_text(log)
    assert r.returncode == 0, log[-4000:]
    # the reference's own debug / progress lines (task.py:104-113, :120, :146, :150)
    assert "Arg - multiprocessing_distributed=True" in log
    assert "GPU x WORLD SIZE = 1" in log
    assert "Process group initialized" in log
    m = json.loads((tmp_path / "metrics.json").read_text())
    assert m["world_size"] == 1 and m["epochs"] == 2 and m["backend"] == "nccl", m
    sd = torch.load(out / "resnet_distributed.pth", weights_only=True, map_location="cpu")
    assert all(k.startswith("module.") for k in sd), list(sd)[:3]
    from mipipe.models.reference import ref_resnet
    tv = ref_resnet("resnet18")  # torchvision's resnet18 module tree, plain torch
    tv.load_state_dict({k[len("module."):]: v for k, v in sd.items()}, strict=True)
