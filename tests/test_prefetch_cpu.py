"""The GEMM operand prefetch's bookkeeping (mipipe/ops/prefetch.py) on the CPU: a step is
recorded between two step boundaries, replayed from the next, a per-step weight operand becomes
a volatile (never warmed) slot, and a different GEMM sequence disarms it until a new recording.
The warming itself needs GPU tensors (tests/test_prefetch_gpu.py); here ``enabled`` is on but the
tensors are CPU ones, so before_weight_gemm returns None while the bookkeeping runs."""
import pytest
import torch

from mipipe.ops import prefetch


@pytest.fixture(autouse=True)
def _reset():
    prefetch.reset()
    yield
    prefetch.reset()


def _step(ws):
    prefetch.step_boundary()
    for w in ws:
        assert prefetch.before_weight_gemm(w) is None  # CPU tensors: never a warm list


def test_record_then_replay():
    ws = [torch.zeros(4, 8), torch.zeros(8, 8), torch.zeros(8, 2)]
    _step(ws)  # first boundary starts the recording
    assert prefetch._S.recording and len(prefetch._S.order) == 3
    _step(ws)  # the second arms it and replays
    assert prefetch._S.armed and prefetch._S.cursor == 3
    _step(ws)
    assert prefetch._S.armed and prefetch._S.cursor == 3 and not prefetch._S.volatile


def test_per_step_operand_is_volatile():
    a, c = torch.zeros(4, 8), torch.zeros(8, 2)
    _step([a, torch.zeros(8, 8), c])
    _step([a, torch.zeros(8, 8), c])  # a new tensor of the same shape in slot 1
    assert prefetch._S.armed and prefetch._S.volatile == {1}


def test_different_sequence_disarms_and_rerecords():
    ws = [torch.zeros(4, 8), torch.zeros(8, 8)]
    _step(ws)
    _step(ws)
    assert prefetch._S.armed
    prefetch.before_weight_gemm(torch.zeros(3, 3))  # an extra GEMM (an evaluation pass)
    assert not prefetch._S.armed and prefetch._S.order == []
    _step(ws)  # records again
    _step(ws)
    assert prefetch._S.armed and prefetch._S.cursor == 2


def test_disabled_mode_still_keeps_the_order(monkeypatch):
    monkeypatch.setattr(prefetch, "_MODE", "0")
    ws = [torch.zeros(4, 8), torch.zeros(8, 8)]
    _step(ws)
    _step(ws)
    assert not prefetch.enabled() and prefetch._S.armed


def test_new_flat_space_and_moved_weights_rerecord():
    from mipipe.optim.flat import FlatParamSpace
    ws = [torch.zeros(4, 8), torch.zeros(8, 8), torch.zeros(8, 2)]
    _step(ws)
    _step(ws)
    assert prefetch._S.armed
    FlatParamSpace([torch.nn.Parameter(torch.zeros(3))])  # another model's optimizer
    assert not prefetch._S.armed and prefetch._S.order == []
    _step(ws)
    _step(ws)
    assert prefetch._S.armed
    # the same shapes at new addresses (another model): most slots move -> record again
    _step([torch.zeros(4, 8), torch.zeros(8, 8), torch.zeros(8, 2)])
    assert not prefetch._S.armed and prefetch._S.order == []
