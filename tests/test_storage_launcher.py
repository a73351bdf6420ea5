"""Local gs:// object store, Google-client aliases, launcher env contract and fail-fast."""
import os
import sys
import time

import pytest

from mipipe.launch import LaunchSpec, build_envs, launch
from mipipe.storage import gcs


def test_gcs_roundtrip(gcs_root, tmp_path):
    c = gcs.Client()
    b = c.bucket("test-pkl")
    b.blob("a/b.txt").upload_from_string("hello")
    assert gcs.uri_to_local_path("gs://test-pkl/a/b.txt") == str(gcs_root / "test-pkl" / "a" / "b.txt")
    assert gcs.uri_to_local_path("/gcs/test-pkl/a/b.txt") == gcs.uri_to_local_path("gs://test-pkl/a/b.txt")
    dst = tmp_path / "x" / "y.txt"
    b.blob("a/b.txt").download_to_filename(str(dst))
    assert dst.read_text() == "hello"
    blob = gcs.blob.Blob.from_string("gs://test-pkl/model/m.pth", client=gcs.Client())
    blob.upload_from_filename(str(dst))
    assert [x.name for x in c.list_blobs("test-pkl")] == ["a/b.txt", "model/m.pth"]
    assert gcs.local_path_to_uri(str(gcs_root / "test-pkl" / "a")) == "gs://test-pkl/a"
    with pytest.raises(FileNotFoundError):
        b.blob("missing").download_to_filename(str(tmp_path / "m"))


def test_google_alias():
    from mipipe.storage import install_google_cloud_alias
    install_google_cloud_alias()
    from google.cloud import storage, aiplatform  # noqa: F401
    from google.cloud.aiplatform import gapic as aip
    assert storage.Client is gcs.Client
    assert aip.AcceleratorType.NVIDIA_TESLA_V100.name == "NVIDIA_TESLA_V100"


def test_env_contract(monkeypatch):
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    monkeypatch.delenv("MIPIPE_GPU_VISIBILITY", raising=False)
    envs = build_envs(LaunchSpec(command=["x"], replica_count=3, accelerator_count=2,
                                 model_dir="gs://b/m/"))
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert all(e["WORLD_SIZE"] == "3" for e in envs)
    # default (replicas share the node): each replica SEES only its own slice, like a Vertex VM
    assert [e["HIP_VISIBLE_DEVICES"] for e in envs] == ["0,1", "2,3", "4,5"]
    assert [(e["MIPIPE_DEVICE_OFFSET"], e["MIPIPE_LOCAL_GPUS"]) for e in envs] == \
        [("0", "2"), ("0", "2"), ("0", "2")]
    assert all(e["AIP_MODEL_DIR"] == "gs://b/m/" for e in envs)
    assert all(e["MASTER_ADDR"] == "127.0.0.1" for e in envs)
    assert len({e["MASTER_PORT"] for e in envs}) == 1
    # opt-in "all": every replica sees the whole node (RCCL xGMI P2P) and owns a slice of it
    envs = build_envs(LaunchSpec(command=["x"], replica_count=3, accelerator_count=2,
                                 gpu_visibility="all"))
    assert all(e["HIP_VISIBLE_DEVICES"] == "0,1,2,3,4,5,6,7" for e in envs)
    assert [(e["MIPIPE_DEVICE_OFFSET"], e["MIPIPE_LOCAL_GPUS"]) for e in envs] == \
        [("0", "2"), ("2", "2"), ("4", "2")]
    monkeypatch.setenv("MIPIPE_GPU_VISIBILITY", "all")
    assert build_envs(LaunchSpec(command=["x"], replica_count=3, accelerator_count=2))[1][
        "MIPIPE_DEVICE_OFFSET"] == "2"
    monkeypatch.delenv("MIPIPE_GPU_VISIBILITY")
    envs = build_envs(LaunchSpec(command=["x"], replica_count=2, accelerator_count=4,
                                 nproc_per_node=4))
    assert [e["RANK"] for e in envs] == [str(i) for i in range(8)]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"] * 2
    # two replicas x 4 GPUs own the whole node: nothing to hide, xGMI P2P between all ranks
    assert envs[5]["HIP_VISIBLE_DEVICES"] == "0,1,2,3,4,5,6,7"
    assert envs[5]["MIPIPE_DEVICE_OFFSET"] == "4" and envs[5]["LOCAL_RANK"] == "1"  # -> cuda:5
    envs = build_envs(LaunchSpec(command=["x"], replica_count=1, accelerator_count=2,
                                 nproc_per_node=2))
    assert [e["HIP_VISIBLE_DEVICES"] for e in envs] == ["0,1", "0,1"]
    cpu = build_envs(LaunchSpec(command=["x"], replica_count=2, accelerator_count=0))
    assert all(e["MIPIPE_FORCE_CPU"] == "1" and e["HIP_VISIBLE_DEVICES"] == "" for e in cpu)
    with pytest.raises(ValueError):
        build_envs(LaunchSpec(command=["x"], replica_count=1, accelerator_count=2,
                              gpu_visibility="some"))


def test_env_slice_from_rocr_visible_devices(monkeypatch):
    """Ids read from ROCR_VISIBLE_DEVICES (Slurm's mask) are physical: HIP renumbers the
    ROCR-filtered set from 0, so HIP_VISIBLE_DEVICES=4,5 under ROCR=4,5,6,7 would name devices
    that do not exist.  The slice narrows ROCR_VISIBLE_DEVICES itself; "all" mode keeps the mask
    and names the slice by positional offsets."""
    for v in ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "MIPIPE_GPU_VISIBILITY"):
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "4,5,6,7")
    envs = build_envs(LaunchSpec(command=["x"], replica_count=2, accelerator_count=1))
    assert [e["ROCR_VISIBLE_DEVICES"] for e in envs] == ["4", "5"]
    assert all("HIP_VISIBLE_DEVICES" not in e and "CUDA_VISIBLE_DEVICES" not in e for e in envs)
    assert all(e["MIPIPE_DEVICE_OFFSET"] == "0" for e in envs)
    envs = build_envs(LaunchSpec(command=["x"], replica_count=2, accelerator_count=2,
                                 gpu_visibility="slice"))
    assert [e["ROCR_VISIBLE_DEVICES"] for e in envs] == ["4,5", "6,7"]
    envs = build_envs(LaunchSpec(command=["x"], replica_count=2, accelerator_count=2,
                                 gpu_visibility="all"))
    assert all(e["ROCR_VISIBLE_DEVICES"] == "4,5,6,7" for e in envs)
    assert [e["MIPIPE_DEVICE_OFFSET"] for e in envs] == ["0", "2"]  # positional: cuda:0 / cuda:2
    # HIP ids under a ROCR mask are already relative to it: the HIP variable is narrowed
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    envs = build_envs(LaunchSpec(command=["x"], replica_count=2, accelerator_count=1))
    assert [e["HIP_VISIBLE_DEVICES"] for e in envs] == ["0", "1"]
    assert all(e["ROCR_VISIBLE_DEVICES"] == "4,5,6,7" for e in envs)


def test_device_count_worker_stays_on_its_slice(tmp_path, monkeypatch):
    """The unmodified reference task.py sizes its mp.spawn by torch.cuda.device_count()
    (task.py:102); under the default visibility every replica of the 3 x 2 topology must count
    exactly its 2 GPUs and no two replicas may share one.  (No GPU here: the worker counts the
    devices HIP would enumerate from its HIP_VISIBLE_DEVICES.)  mipipe's own consumers name the
    same slice through local_device_ids()."""
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3,4,5,6,7")
    monkeypatch.delenv("MIPIPE_GPU_VISIBILITY", raising=False)
    out = tmp_path / "out"
    out.mkdir()
    script = tmp_path / "w.py"
    script.write_text(
        "import os, sys\n"
        "vis = [v for v in os.environ['HIP_VISIBLE_DEVICES'].split(',') if v]\n"
        "ngpus_per_node = len(vis)  # what torch.cuda.device_count() returns under it\n"
        "from mipipe.launch.env import local_device_ids\n"
        "own = [vis[i] for i in local_device_ids()]\n"
        f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write("
        "f'{ngpus_per_node} ' + ','.join(own))\n")
    rc = launch(LaunchSpec(command=[sys.executable, str(script)], replica_count=3,
                           accelerator_count=2, echo=False,
                           env={"PYTHONPATH": os.path.dirname(os.path.dirname(__file__))}))
    assert rc == 0
    got = [(out / str(r)).read_text().split() for r in range(3)]
    assert [int(g[0]) for g in got] == [2, 2, 2]
    assert [g[1] for g in got] == ["0,1", "2,3", "4,5"]


def test_launchers_share_one_env_builder(monkeypatch):
    """bench.py's launcher (launch.local.rank_envs) and the job launcher (launch.build_envs) build
    rank environments with the same function: same RCCL settings, same visibility policy."""
    from mipipe.launch.local import rank_envs
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0,1,2,3")
    monkeypatch.setenv("MIPIPE_RCCL_PROFILE", "overlap")
    a = rank_envs(4, port=23456)
    b = build_envs(LaunchSpec(command=["x"], replica_count=1, accelerator_count=4,
                              nproc_per_node=4, master_port=23456))
    for ea, eb in zip(a, b):
        for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_PORT",
                  "HIP_VISIBLE_DEVICES", "HSA_ENABLE_IPC_MODE_LEGACY", "TORCH_NCCL_HIGH_PRIORITY",
                  "NCCL_MAX_NCHANNELS"):
            assert ea.get(k) == eb.get(k), k
    from mipipe.launch.env import device_offset
    assert [int(e["LOCAL_RANK"]) + device_offset(e) for e in b] == [0, 1, 2, 3]
    with pytest.raises(RuntimeError):
        build_envs(LaunchSpec(command=["x"], replica_count=5, accelerator_count=2))


def test_fail_fast(tmp_path):
    script = tmp_path / "s.py"
    script.write_text(
        "import os, sys, time\n"
        "r = int(os.environ['RANK'])\n"
        "if r == 1:\n    time.sleep(0.3); sys.exit(7)\n"
        "time.sleep(60)\n")
    t0 = time.time()
    rc = launch(LaunchSpec(command=[sys.executable, str(script)], replica_count=3, echo=False,
                           grace_period=2.0, log_dir=str(tmp_path / "logs")))
    assert rc == 7
    assert time.time() - t0 < 20
    assert (tmp_path / "logs" / "rank0.log").exists()


def test_timeout(tmp_path):
    script = tmp_path / "s.py"
    script.write_text("import time\ntime.sleep(60)\n")
    rc = launch(LaunchSpec(command=[sys.executable, str(script)], echo=False, timeout=1.0,
                           grace_period=1.0))
    assert rc == 124


def test_dotenv_and_pipeline_config(tmp_path):
    """Notebook driver config (nb:73-86): .env parsing + PIPELINE_ROOT derivation."""
    from mipipe.utils import load_dotenv, parse_dotenv, pipeline_config
    p = tmp_path / ".env"
    p.write_text('# comment\nPROJECT_ID=my-proj\nexport BUCKET="my-bucket"  \n'
                 "ROOT=gs://${BUCKET}/x # trailing comment\nRAW='${BUCKET}'\nEMPTY=\n")
    env = {"BUCKET": "preset"}
    vals = load_dotenv(str(p), environ=env)
    assert vals["ROOT"] == "gs://my-bucket/x" and vals["RAW"] == "${BUCKET}" and vals["EMPTY"] == ""
    assert env["BUCKET"] == "preset" and env["PROJECT_ID"] == "my-proj"  # existing vars win
    load_dotenv(str(p), override=True, environ=env)
    assert env["BUCKET"] == "my-bucket"
    cfg = pipeline_config(env)
    assert (cfg.project_id, cfg.bucket, cfg.region) == ("my-proj", "my-bucket", "us-central1")
    assert cfg.pipeline_root == "gs://my-bucket/pipeline_root"
    assert load_dotenv(str(tmp_path / "missing.env"), environ={}) == {}
    assert parse_dotenv('A="x\\ny"', {})["A"] == "x\ny"
