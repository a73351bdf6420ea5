"""Native host runtime (csrc/runtime): process supervisor, DAG scheduler, record loader —
each checked against its pure-Python twin / definition."""
import os
import random
import sys
import time

import numpy as np
import pytest
import torch

from mipipe.runtime import runtime, runtime_available
from mipipe.orchestrator.runner import _PyDag
from mipipe.data import records as R

native = pytest.mark.skipif(not runtime_available(), reason="mipipe._runtime not built")


@native
def test_process_group_fail_fast_and_logs(tmp_path):
    rt = runtime()
    pg = rt.ProcessGroup(echo=False)
    py = sys.executable
    t0 = time.time()
    pg.spawn([py, "-c", "import time; print('ok0', flush=True); time.sleep(30)"], [], "",
             str(tmp_path / "r0.log"), "[r0] ")
    pg.spawn([py, "-c", "import sys, time; time.sleep(0.3); print('boom', flush=True); sys.exit(3)"],
             [], "", str(tmp_path / "r1.log"), "[r1] ")
    rc = pg.wait(60.0, 2.0)
    assert rc == 3 and pg.failed_rank == 1
    assert time.time() - t0 < 20
    codes = pg.exit_codes()
    assert codes[1] == 3 and codes[0] == 128 + 15  # SIGTERMed by fail-fast
    assert "ok0" in (tmp_path / "r0.log").read_text()
    assert "boom" in (tmp_path / "r1.log").read_text()


@native
def test_process_group_timeout_and_env(tmp_path):
    rt = runtime()
    pg = rt.ProcessGroup(echo=False)
    env = [f"{k}={v}" for k, v in os.environ.items()] + ["MIPIPE_T=42"]
    pg.spawn([sys.executable, "-c", "import os; print(os.environ['MIPIPE_T'])"], env, str(tmp_path),
             str(tmp_path / "a.log"), "")
    assert pg.wait(30.0, 1.0) == 0
    assert (tmp_path / "a.log").read_text().strip() == "42"
    pg2 = rt.ProcessGroup(echo=False)
    pg2.spawn([sys.executable, "-c", "import time; time.sleep(30)"], [], "", "", "")
    assert pg2.wait(0.5, 1.0) == 124


def _drive(s, n, fail=(), skip=()):
    order = []
    while True:
        r = s.next_ready()
        s.take_cancelled()
        if not r:
            break
        for i in r:
            order.append(i)
            s.complete(i, 5 if i in fail else (4 if i in skip else 2))
    return order, list(s.states())


@native
def test_dag_scheduler_matches_python_twin():
    rt = runtime()
    rnd = random.Random(0)
    for trial in range(200):
        n = rnd.randint(1, 12)
        deps = [[d for d in range(i) if rnd.random() < 0.3] for i in range(n)]
        always = [rnd.random() < 0.15 for _ in range(n)]
        fail = {i for i in range(n) if rnd.random() < 0.15}
        ff = rnd.random() < 0.5
        a = _drive(rt.DagScheduler(n, deps, always, ff), n, fail)
        b = _drive(_PyDag(n, deps, always, ff), n, fail)
        assert a == b, (deps, always, fail)
        assert all(s >= 2 for s in a[1])


@native
def test_dag_scheduler_semantics():
    rt = runtime()
    D = rt.DagScheduler
    # 0 -> 1 -> 2, 0 -> 3 (exit handler: always runs)
    s = D(4, [[], [0], [1], [0]], [False, False, False, True], True)
    assert s.next_ready() == [0]
    s.complete(0, D.FAILED)
    assert s.next_ready() == [3]
    assert sorted(s.take_cancelled()) == [1, 2]
    s.complete(3, D.SUCCEEDED)
    assert s.finished()
    with pytest.raises(ValueError):
        D(2, [[1], [0]], [False, False], True)


def _write(tmp_path, n=37, shape=(3, 8, 8)):
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(n, *shape), dtype=np.uint8)
    lab = rng.integers(0, 10, size=n)
    f1, f2 = str(tmp_path / "a.bin"), str(tmp_path / "b.bin")
    R.write_records(f1, img[:20], lab[:20])
    R.write_records(f2, img[20:], lab[20:])
    return [f1, f2], img, lab


@pytest.mark.parametrize("train", [False, True])
def test_record_loader_matches_reference_transform(tmp_path, train):
    files, img, lab = _write(tmp_path)
    sampler = R.DistributedSampler(len(lab), num_replicas=2, rank=1, shuffle=True, seed=3)
    dl = R.RecordDataLoader(files, (3, 8, 8), batch_size=5, sampler=sampler, train=train, pad=2,
                            seed=11, workers=3, prefetch=2)
    for epoch in (0, 1):
        dl.set_epoch(epoch)
        idx = list(iter(sampler))
        got_x = torch.cat([x for x, _ in dl])
        got_y = torch.cat([y for _, y in iter(dl)])
        ref = np.stack([R.reference_transform(img[i], i, epoch, 11, train, 2 if train else 0,
                                              train, R.CIFAR10_MEAN, R.CIFAR10_STD) for i in idx])
        assert got_x.shape == ref.shape
        np.testing.assert_allclose(got_x.numpy(), ref, rtol=1e-5, atol=1e-5)
        assert torch.equal(got_y, torch.from_numpy(lab[idx]))


def test_record_loader_python_fallback_agrees(tmp_path, monkeypatch):
    files, img, lab = _write(tmp_path)
    a = R.RecordDataLoader(files, (3, 8, 8), 4, train=True, pad=2, seed=5)
    xa = torch.cat([x for x, _ in a])
    monkeypatch.setenv("MIPIPE_NO_NATIVE_RUNTIME", "1")
    b = R.RecordDataLoader(files, (3, 8, 8), 4, train=True, pad=2, seed=5)
    assert not b.native
    xb = torch.cat([x for x, _ in b])
    np.testing.assert_allclose(xa.numpy(), xb.numpy(), rtol=1e-5, atol=1e-5)


def test_synthetic_dataset_files(tmp_path):
    man = R.write_synthetic_dataset(str(tmp_path), "cifar10", n_train=64, n_test=16)
    x, y = R.read_records(man["files"]["train"], (3, 32, 32))
    assert x.shape == (64, 3, 32, 32) and y.max() < 10
    assert R.dataset_files(str(tmp_path), "cifar10", "test") == [man["files"]["test"]]
