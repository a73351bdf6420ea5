"""bench.py's driver contract on the CPU: `python bench.py --gpus N` spawns its own N ranks
(task.py:117-124's one-process-per-GPU), every rank checks the process-group size, rank 0
prints exactly one JSON line with n_gpus = N.  gloo stands in for RCCL here."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")
CPU_ARGS = ["--device", "cpu", "--model", "mnist_cnn", "--res", "28", "--classes", "10",
            "--batch", "8", "--steps", "2", "--warmup", "1"]


def _env(**kw):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e["OMP_NUM_THREADS"] = "1"  # single-threaded CPU kernels: run-to-run identical sums
    e.update(kw)
    return e


def _json_lines(out: str):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("n", [1, 2])
def test_bench_self_spawn_gloo(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n)] + CPU_ARGS, env=_env(),
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout  # only rank 0 prints to stdout
    j = lines[0]
    assert j["n_gpus"] == n and j["config"]["parallelism"] == f"dp{n}"
    assert j["config"]["global_batch"] == 8 * n
    assert j["steps"] == 2 and j["warmup"] == 1 and j["value"] > 0
    if n > 1:
        from mipipe.ops._native import native_available
        assert j["config"]["native_reducer"] == native_available()
        assert j["config"]["rccl"]["TORCH_NCCL_HIGH_PRIORITY"] == "1"


def test_bench_force_reduce_world1_gloo():
    """--force-reduce wraps in DDP and issues the collectives at world size 1."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--force-reduce"] + CPU_ARGS,
                       env=_env(MASTER_ADDR="127.0.0.1", MASTER_PORT="0", WORLD_SIZE="1",
                                RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    j = _json_lines(r.stdout)[0]
    assert j["config"]["force_reduce"] is True and j["n_gpus"] == 1


def test_bench_rejects_world_mismatch():
    """A launcher that started fewer ranks than --gpus must not yield a silent 1-rank number."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"] + CPU_ARGS,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       capture_output=True, text=True, timeout=120, cwd="/tmp")
    assert r.returncode != 0
    assert _json_lines(r.stdout) == []


def test_spawn_local_ranks_fail_fast(tmp_path):
    from mipipe.launch.local import spawn_local_ranks
    script = tmp_path / "s.py"
    script.write_text(
        "import os, sys, time\n"
        "r = int(os.environ['RANK'])\n"
        "assert os.environ['WORLD_SIZE'] == '3' and os.environ['LOCAL_RANK'] == str(r)\n"
        "if r == 1: sys.exit(7)\n"
        "time.sleep(60)\n")
    import time
    t0 = time.time()
    rc = spawn_local_ranks([sys.executable, str(script)], 3, grace=2.0)
    assert rc == 7
    assert time.time() - t0 < 30  # the sleeping ranks were terminated


def test_spawn_local_ranks_env_contract():
    from mipipe.launch.local import rank_envs
    envs = rank_envs(4, port=12345)
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1"
               and e["MASTER_PORT"] == "12345" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
               for e in envs)


@pytest.mark.parametrize("comm", ["fp32", "bf16"])
def test_bench_world4_gloo_matches_global_batch(tmp_path, comm):
    """`bench.py --gpus 4` (4 gloo ranks, mipipe DDP) ends with bit-identical parameters on
    every rank, equal (to fp32 reduction-order noise) to ONE process that runs the same four
    per-rank batches and averages their gradients (--emulate-ranks 4): the DDP contract of the
    reference's task.py:189 (average of per-rank gradients, rank 0's BN buffers broadcast before
    every forward), rehearsed at world 4 before any 8-GPU run."""
    import torch
    args = ["--device", "cpu", "--model", "mnist_cnn", "--res", "28", "--classes", "10",
            "--batch", "8", "--steps", "3", "--warmup", "1"]
    d4, d1 = tmp_path / "w4", tmp_path / "w1"
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dump-params", str(d4),
                        "--comm-dtype", comm] + args,
                       env=_env(), capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--emulate-ranks", "4",
                        "--dump-params", str(d1)] + args,
                       env=_env(), capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    ranks = [torch.load(d4 / f"rank{i}.pt", weights_only=True) for i in range(4)]
    ref = torch.load(d1 / "rank0.pt", weights_only=True)
    for rk in ranks[1:]:
        for a, b in zip(ranks[0]["params"], rk["params"]):
            assert torch.equal(a, b)
    moved = 0.0
    # fp32 wire: reduction-order noise only (~3e-8): a race between the per-forward buffer
    # broadcast and the BN statistics shift showed up here as 1e-5..2e-4 run-to-run noise.
    # bf16 wire: gradients rounded to 8 bits before the sum; 4 SGD steps at lr 0.1 move a
    # parameter by <= ~1e-3 relative of its update.
    tol = dict(rtol=1e-5, atol=1e-6) if comm == "fp32" else dict(rtol=1e-3, atol=2e-4)
    for a, b in zip(ranks[0]["params"], ref["params"]):
        assert torch.allclose(a, b, **tol), (a - b).abs().max()
        moved += float((a - b).abs().max())
    for a, b in zip(ranks[0]["buffers"], ref["buffers"]):
        btol = dict(rtol=1e-4, atol=1e-5) if comm == "fp32" else dict(rtol=1e-2, atol=1e-3)
        assert torch.allclose(a.float(), b.float(), **btol)


def test_rccl_profiles_env():
    """MIPIPE_RCCL_PROFILE channel profiles: applied as defaults (the environment wins), the
    high-priority comm stream always, unknown names rejected; the settings report lists them."""
    from mipipe.parallel.dist_utils import configure_rccl_env, rccl_settings
    e = configure_rccl_env({})
    assert e["TORCH_NCCL_HIGH_PRIORITY"] == "1" and "NCCL_MAX_NCHANNELS" not in e
    e = configure_rccl_env({"MIPIPE_RCCL_PROFILE": "overlap"})
    assert e["NCCL_MAX_NCHANNELS"] == "8"
    e = configure_rccl_env({"NCCL_MIN_NCHANNELS": "4"}, profile="bandwidth")
    assert e["NCCL_MIN_NCHANNELS"] == "4"  # explicit setting kept
    with pytest.raises(ValueError):
        configure_rccl_env({}, profile="fastest")
    rep = rccl_settings({"NCCL_MIN_NCHANNELS": "32", "PATH": "/bin", "TORCH_NCCL_HIGH_PRIORITY": "1"})
    assert rep == {"NCCL_MIN_NCHANNELS": "32", "TORCH_NCCL_HIGH_PRIORITY": "1"}


def test_bench_world4_gloo_bert_matches_emulated_ranks(tmp_path):
    """`bench.py --gpus 4 --model bert_tiny` (4 gloo ranks, mipipe DDP with the tied word
    embedding's lookup gradient exchanged as sparse (id, row) pairs) ends with bit-identical
    parameters on every rank, equal to one process that runs the four per-rank batches and
    averages their gradients (--emulate-ranks 4)."""
    import torch
    args = ["--device", "cpu", "--model", "bert_tiny", "--batch", "2", "--seq", "32",
            "--steps", "2", "--warmup", "1", "--bert-dropout", "0"]
    d4, d1 = tmp_path / "w4", tmp_path / "w1"
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dump-params", str(d4)] + args,
                       env=_env(), capture_output=True, text=True, timeout=900, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--emulate-ranks", "4",
                        "--dump-params", str(d1)] + args,
                       env=_env(), capture_output=True, text=True, timeout=900, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    ranks = [torch.load(d4 / f"rank{i}.pt", weights_only=True) for i in range(4)]
    ref = torch.load(d1 / "rank0.pt", weights_only=True)
    for rk in ranks[1:]:
        for a, b in zip(ranks[0]["params"], rk["params"]):
            assert torch.equal(a, b)
    for a, b in zip(ranks[0]["params"], ref["params"]):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6), (a - b).abs().max()


def test_bench_reference_config_block_gloo():
    """`--reference-config on` times the reference's config of record (ResNet-18 32x32, 1000
    classes, fp32, deterministic) after the headline in the same process (and, here, under a
    2-rank gloo DDP), and reports it inside the ONE JSON line."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--reference-config", "on",
                        "--time-deterministic", "on", "--ref-batch", "4"] + CPU_ARGS, env=_env(),
                       capture_output=True, text=True, timeout=600, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    j = lines[0]
    assert j["config"]["model"] == "mnist_cnn" and j["n_gpus"] == 2
    ref = j["reference_config"]
    assert ref["model"] == "resnet18" and ref["classes"] == 1000 and ref["image_size"] == 32
    assert ref["dtype"] == "fp32" and ref["deterministic"] is True
    assert ref["batch_per_gpu"] == 4 and ref["global_batch"] == 8
    assert ref["value"] > 0 and ref["ms_per_step"] > 0 and ref["steps"] == 2
    det = j["deterministic_variant"]
    assert det["deterministic"] is True and det["value"] > 0 and det["steps"] == 2
    assert j["config"]["deterministic"] is False
