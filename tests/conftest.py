import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

# Under pytest-xdist every worker would otherwise start one intra-op thread per CPU; the
# oversubscribed OpenMP pools turn a 1.4 s fp64 parity test into minutes.  Split the CPUs.
_nworkers = int(os.environ.get("PYTEST_XDIST_WORKER_COUNT", "1") or 1)
if _nworkers > 1:
    import torch
    torch.set_num_threads(max(1, (os.cpu_count() or 1) // _nworkers))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture
def gcs_root(tmp_path, monkeypatch):
    root = tmp_path / "gcs"
    root.mkdir()
    monkeypatch.setenv("MIPIPE_GCS_ROOT", str(root))
    monkeypatch.setenv("MIPIPE_CACHE_DIR", str(tmp_path / "cache"))
    return root


def cuda_ok():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
