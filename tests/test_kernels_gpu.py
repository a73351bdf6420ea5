"""Numerics of every gfx950 HIP kernel vs the plain-PyTorch fp32 reference of the same op.

Inputs are random (never zeros; cdna guide rule 25); bf16 inputs are quantised first so both
sides see identical operands; tolerances are relative to the output magnitude.
Run on an MI355X:  python -m pytest tests -m gpu
"""
import math

import pytest
import torch

from mipipe.ops import _ref
from mipipe.ops._native import native, native_available

pytestmark = pytest.mark.gpu

dev = "cuda"


def _skip_no_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    assert native_available(), "mipipe._C must be built for GPU tests (no silent fallback)"


@pytest.fixture(autouse=True)
def _gpu():
    _skip_no_gpu()
    torch.manual_seed(1234)
    yield


def rel_err(a, b):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    return ((a - b).abs().max() / (b.abs().max() + 1e-6)).item()


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def rnd(dt, *shape, scale=1.0):
    """Random operand in the kernel dtype (bf16 inputs are quantised before the reference)."""
    return (torch.randn(*shape, device=dev) * scale).to(dt)


# tolerances per operand dtype: bf16 outputs / fp32 accumulation of bf16 products / fp32 (the
# reference's precision: split-bf16x3 main loop, ~1e-6 measured)
TOL_OUT = {torch.bfloat16: 1e-2, torch.float32: 1e-4}
TOL_ACC = {torch.bfloat16: 2e-3, torch.float32: 1e-4}
TOL_WGRAD = {torch.bfloat16: 5e-3, torch.float32: 1e-4}
DTYPES = pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32], ids=["bf16", "fp32"])


def hi_ref(t):
    """Reference operand: float64 on the CPU for fp32 kernels (MIOpen has no float64 conv),
    fp32 on the GPU for bf16 kernels."""
    return t.detach().double().cpu() if t.dtype in (torch.float32, torch.float64) else t.float()


CONV_CASES = [
    # N, H, W, Ci, Co, k, s, p
    (2, 8, 8, 64, 64, 3, 1, 1),
    (2, 9, 7, 32, 72, 3, 1, 1),
    (2, 16, 16, 64, 256, 1, 1, 0),
    (2, 16, 16, 256, 64, 1, 1, 0),
    (2, 16, 16, 128, 128, 3, 2, 1),
    (2, 16, 16, 256, 512, 1, 2, 0),
    (2, 32, 32, 8, 64, 7, 2, 3),
    (3, 7, 7, 512, 512, 3, 1, 1),
    (1, 5, 5, 24, 40, 3, 1, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd(case):
    N, H, W, Ci, Co, k, s, p = case
    x = bf(N, H, W, Ci)
    w = bf(Co, k, k, Ci, scale=1.0 / math.sqrt(Ci * k * k))
    shift = torch.randn(Co, device=dev) * 0.1
    y, ps, pss = native().conv_fwd(x, w, s, p, shift)
    yr, psr, pssr = _ref.conv_fwd(x.float(), w.float(), s, p, shift)
    assert y.shape == yr.shape
    assert rel_err(y, yr) < 1e-2
    assert rel_err(ps.sum(0), psr[0]) < 2e-3
    assert rel_err(pss.sum(0), pssr[0]) < 2e-3
    y2, a, b = native().conv_fwd(x, w, s, p, None)
    assert a is None and torch.equal(y, y2)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_dgrad(case):
    N, H, W, Ci, Co, k, s, p = case
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = bf(N, Ho, Wo, Co)
    w = bf(Co, k, k, Ci, scale=1.0 / math.sqrt(Co * k * k))
    dx = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p)
    dxr = _ref.conv_dgrad(dy.float(), w.float(), (N, H, W, Ci), s, p)
    assert rel_err(dx, dxr) < 1e-2


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_wgrad(case):
    N, H, W, Ci, Co, k, s, p = case
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = bf(N, Ho, Wo, Co)
    x = bf(N, H, W, Ci)
    dw = native().conv_wgrad(dy, x, k, k, s, p)
    dwr = _ref.conv_wgrad(dy.float(), x.float(), k, k, s, p)
    assert dw.dtype == torch.float32 and dw.shape == dwr.shape
    assert rel_err(dw, dwr) < 5e-3


@pytest.mark.parametrize("shape", [(8, 28, 28, 64, 64, 3, 1, 1), (4, 14, 14, 256, 512, 3, 1, 1),
                                   (4, 17, 17, 96, 40, 3, 1, 1), (2, 12, 12, 64, 64, 5, 1, 2),
                                   (8, 56, 56, 128, 128, 3, 2, 1), (4, 15, 15, 64, 96, 3, 2, 1),
                                   (2, 20, 20, 64, 64, 5, 2, 2)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float32])
def test_conv_fwd_writes_dgrad_flipped_weight(shape, dt):
    """conv_fwd(wflip=buf) writes the tap-flipped (per stride-parity class) sub-kernels in extra
    blocks of the same launch; conv_dgrad(wflip_pre=buf) then skips its flip kernels: y
    unchanged, dx bit-identical to the self-flipping data-grad, and both against the fp32
    reference (stride 1 and 2)."""
    N, H, W, Ci, Co, k, s, p = shape
    C = native()
    if not C.dgrad_preflip_ok([N, H, W, Ci], [Co, k, k, Ci], s, p):
        pytest.skip("not a forward-style stride-1 data-grad shape")
    x = torch.randn(N, H, W, Ci, device=dev).to(dt)
    w = (torch.randn(Co, k, k, Ci, device=dev) * 0.05).to(dt)
    buf = torch.full((w.numel(),), float("nan"), device=dev).to(dt)
    y0 = C.conv_fwd(x, w, s, p)[0]
    y1 = C.conv_fwd(x, w, s, p, wflip=buf)[0]
    assert torch.equal(y0, y1)
    assert not torch.isnan(buf.float()).any()
    Ho = (H + 2 * p - k) // s + 1
    dy = torch.randn(N, Ho, Ho, Co, device=dev).to(dt)
    dx0 = C.conv_dgrad(dy, w, [N, H, W, Ci], s, p)
    dx1 = C.conv_dgrad(dy, w, [N, H, W, Ci], s, p, wflip_pre=buf)
    assert torch.equal(dx0, dx1)
    dxr = _ref.conv_dgrad(dy.float(), w.float(), (N, H, W, Ci), s, p)
    assert rel_err(dx1, dxr) < (1e-2 if dt == torch.bfloat16 else 1e-4)


@pytest.mark.parametrize("shape", [(32, 14, 14, 256, 1024, 1, 1, 0), (16, 28, 28, 64, 64, 3, 1, 1),
                                   (16, 56, 56, 64, 128, 3, 2, 1)])
@DTYPES
def test_conv_wgrad_workspace_plans(shape, dt):
    """Workspace split-K weight-grad plans (flag 1024: per-split slices + ordered sum instead of
    fp32 atomics) against the fp32 reference, accumulating into an existing gradient, for
    every tile and the split counts the tuner tries (incl. 3 / 6 / 12 / 24); bit-identical
    reruns.  fp32 operands run the split-bf16x3 main loop (tiles 0 / 2 / 8; others resolve to
    the default) and must stay within fp32-class error."""
    N, H, W, Ci, Co, k, s, p = shape
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy, x = rnd(dt, N, Ho, Wo, Co), rnd(dt, N, H, W, Ci)
    dwr = _ref.conv_wgrad(hi_ref(dy), hi_ref(x), k, k, s, p)
    base = torch.randn(dwr.shape, device=dev)
    cfgs = (0, 2, 8) if dt == torch.float32 else (0, 2, 9)
    for cfg in cfgs:
        for sp in (3, 4, 6, 12, 16, 24, 32):
            plan = (cfg + 16 * sp) | 1024
            out = base.clone()
            native().conv_wgrad(dy, x, k, k, s, p, out, cfg=plan)
            assert rel_err(hi_ref(out) - hi_ref(base), dwr) < TOL_WGRAD[dt], (cfg, sp)
            out2 = base.clone()
            native().conv_wgrad(dy, x, k, k, s, p, out2, cfg=plan)
            assert torch.equal(out, out2), (cfg, sp)


def test_conv_wgrad_large_k_splitk():
    # K = N*Ho*Wo large enough to exercise split-K atomics
    x = bf(16, 28, 28, 64)
    dy = bf(16, 28, 28, 64)
    dw = native().conv_wgrad(dy, x, 3, 3, 1, 1)
    dwr = _ref.conv_wgrad(dy.float(), x.float(), 3, 3, 1, 1)
    assert rel_err(dw, dwr) < 5e-3


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (300, 72, 200), (64, 1000, 2048),
                                   (1024, 768, 768), (40, 3072, 768)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
def test_gemm(M, N, K, ta, tb):
    if (ta and M % 8) or (not ta and K % 8) or N % 8:
        pytest.skip("layout constraint")
    if tb and K % 8:
        pytest.skip("layout constraint")
    a = bf(K, M) if ta else bf(M, K)
    b = bf(N, K) if tb else bf(K, N)
    bias = torch.randn(N, device=dev)
    out = native().gemm(a, b, ta, tb, bias, "relu", torch.bfloat16, None, 0.0)
    ref = _ref.gemm(a.float(), b.float(), ta, tb, bias, "relu", torch.float32)
    assert rel_err(out, ref) < 1e-2
    out32 = native().gemm(a, b, ta, tb, None, "none", torch.float32, None, 0.0)
    ref32 = _ref.gemm(a.float(), b.float(), ta, tb, None, "none", torch.float32)
    assert rel_err(out32, ref32) < 2e-3
    acc = torch.randn(M, N, device=dev)
    acc0 = acc.clone()
    native().gemm(a, b, ta, tb, None, "none", torch.float32, acc, 1.0)
    assert rel_err(acc, acc0 + ref32) < 2e-3


@pytest.mark.parametrize("M,N,K", [(1024, 768, 768), (300, 72, 200), (768, 256, 4096)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False)])
@DTYPES
def test_gemm_every_plan(M, N, K, ta, tb, dt):
    """Every (tile config x split-K) plan of the GEMM gives the same product: activation-dtype
    output with the bias / ReLU epilogue, and fp32 accumulation into C (split-K atomics, the
    non-atomic read-modify-write of splits == 1, and workspace split-K: slices + ordered sum).
    fp32 operands (split-bf16x3) against a float64 reference at 1e-4."""
    if (ta and M % 8) or (not ta and K % 8) or N % 8:
        pytest.skip("layout constraint")
    a = rnd(dt, K, M) if ta else rnd(dt, M, K)
    b = rnd(dt, N, K) if tb else rnd(dt, K, N)
    bias = torch.randn(N, device=dev)
    ref = _ref.gemm(a.double(), b.double(), ta, tb, bias.double(), "relu", torch.float64)
    ref32 = _ref.gemm(a.double(), b.double(), ta, tb, None, "none", torch.float64)
    for cfg in range(native().CONV_TILE_CONFIGS):
        out = native().gemm(a, b, ta, tb, bias, "relu", dt, None, 0.0, cfg)
        assert out.dtype == dt and rel_err(out, ref) < TOL_OUT[dt], cfg
        for sp in (1, 2, 3, 4):
            acc = torch.randn(M, N, device=dev)
            acc0 = acc.clone()
            native().gemm(a, b, ta, tb, None, "none", torch.float32, acc, 1.0, cfg + 16 * sp)
            assert rel_err(acc.double() - acc0.double(), ref32) < TOL_ACC[dt], (cfg, sp)
        for sp in (2, 3, 4, 6, 8, 12, 24):  # workspace split-K (kPlanWs): slices + ordered sum
            acc = torch.randn(M, N, device=dev)
            acc0 = acc.clone()
            native().gemm(a, b, ta, tb, None, "none", torch.float32, acc, 1.0,
                          (cfg + 16 * sp) | 1024)
            assert rel_err(acc.double() - acc0.double(), ref32) < TOL_ACC[dt], (cfg, sp, "ws")
            acc2 = acc0.clone()
            native().gemm(a, b, ta, tb, None, "none", torch.float32, acc2, 1.0,
                          (cfg + 16 * sp) | 1024)
            assert torch.equal(acc, acc2), (cfg, sp, "ws split-K must be deterministic")


@pytest.mark.parametrize("M,N,K", [(1024, 1000, 512), (1024, 512, 1000), (200, 136, 264)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False)])
def test_gemm_splitk_fp32_output(M, N, K, ta, tb):
    """Workspace split-K plans of an fp32-output GEMM (the reference config's fc layer: 64-128
    output tiles for 256 CUs): slices summed in order with the bias by one pass — every fp32 tile
    at 2/3/4/8 splits against a float64 reference at 1e-4, bit-identical reruns."""
    if N % 8:
        pytest.skip("layout constraint")
    a = torch.randn(M, K, device=dev)
    b = torch.randn(N, K, device=dev) if tb else torch.randn(K, N, device=dev)
    bias = torch.randn(N, device=dev)
    ref = _ref.gemm(a.double().cpu(), b.double().cpu(), ta, tb, bias.double().cpu(), "none",
                    torch.float64)
    for cfg in (0, 2, 8):
        for sp in (2, 3, 4, 8):
            plan = (cfg + 16 * sp) | 1024
            out = native().gemm(a, b, ta, tb, bias, "none", torch.float32, None, 0.0, plan)
            assert out.dtype == torch.float32 and rel_err(out, ref) < 1e-4, (cfg, sp)
            out2 = native().gemm(a, b, ta, tb, bias, "none", torch.float32, None, 0.0, plan)
            assert torch.equal(out, out2), (cfg, sp)


@pytest.mark.parametrize("M,N,K", [(512, 768, 8192), (200, 136, 4104), (640, 768, 30528)])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False)])
def test_gemm_splitk_bf16_output(M, N, K, ta, tb):
    """Workspace split-K plans (flag 1024) of a bf16-output GEMM (e.g. the MLM decoder data-grad,
    K = 30528): every split stores its own fp32 slice, one pass adds the slices (and the bias) in
    order and rounds to bf16 — every tile config at 2/4/8 splits against the fp32 product, with
    and without a bias; deterministic (bit-identical reruns)."""
    a = bf(M, K)
    b = bf(N, K) if tb else bf(K, N)
    bias = torch.randn(N, device=dev)
    ref = _ref.gemm(a.float(), b.float(), ta, tb, None, "none", torch.float32)
    for cfg in range(native().CONV_TILE_CONFIGS):
        for sp in (2, 4, 8):
            plan = (cfg + 16 * sp) | 1024
            out = native().gemm(a, b, ta, tb, None, "none", torch.bfloat16, None, 0.0, plan)
            assert out.dtype == torch.bfloat16 and out.shape == (M, N)
            assert rel_err(out, ref) < 1e-2, (cfg, sp)
            ob = native().gemm(a, b, ta, tb, bias, "none", torch.bfloat16, None, 0.0, plan)
            assert rel_err(ob, ref + bias) < 1e-2, (cfg, sp, "bias")
            assert torch.equal(ob, native().gemm(a, b, ta, tb, bias, "none", torch.bfloat16,
                                                 None, 0.0, plan)), (cfg, sp, "deterministic")


@pytest.mark.parametrize("M,N,K", [(1024, 768, 768), (4096, 768, 3072), (200, 64, 136)])
def test_gemm_addend_epilogue(M, N, K):
    """dx = dy @ W + addend in one GEMM (the residual-stream gradient fused into the data-grad
    epilogue), for every tile config."""
    a, b, add = bf(M, K), bf(K, N, scale=0.05), bf(M, N)
    ref = a.float() @ b.float() + add.float()
    for cfg in range(native().CONV_TILE_CONFIGS):
        out = native().gemm(a, b, False, False, None, "none", torch.bfloat16, None, 0.0, cfg, add)
        assert rel_err(out, ref) < 1e-2, cfg
        if K >= 1024:  # workspace split-K: the ordered slice sum adds the addend
            for sp in (3, 6):
                plan = (cfg + 16 * sp) | 1024
                ow = native().gemm(a, b, False, False, None, "none", torch.bfloat16, None, 0.0,
                                   plan, add)
                assert rel_err(ow, ref) < 1e-2, (cfg, sp, "ws")
                assert torch.equal(ow, native().gemm(a, b, False, False, None, "none",
                                                     torch.bfloat16, None, 0.0, plan, add))


@pytest.mark.parametrize("M,N,K,ta,tb,mode", [
    (768, 3072, 4096, True, False, 2), (2304, 768, 4096, True, False, 2),
    (200, 136, 4104, True, False, 2), (640, 768, 30528, False, True, 0),
    (4096, 768, 3072, False, False, 3), (1000, 776, 2048, False, True, 0)])
def test_gemm_ws_finish_in_kernel_matches_slice_sum(M, N, K, ta, tb, mode):
    """Workspace split-K finished inside the GEMM (the last split of each tile sums the slices,
    WsFinish) == the separate ordered slice-sum kernel, bit for bit, for every tile config and
    2..8 splits (the separate fp32 sum of >= 8 slices runs a strided order: there equal to fp32
    rounding); repeated launches give bit-identical results (the self-resetting tickets), also
    replayed from a graph."""
    C = native()
    a = bf(K, M) if ta else bf(M, K)
    b = bf(N, K, scale=0.05) if tb else bf(K, N, scale=0.05)
    bias = torch.randn(N, device=dev) if mode == 0 else None
    add = bf(M, N) if mode == 3 else None
    acc0 = torch.randn(M, N, device=dev)

    def run(plan):
        if mode == 2:
            acc = acc0.clone()
            C.gemm(a, b, ta, tb, None, "none", torch.float32, acc, 1.0, plan)
            return acc
        return C.gemm(a, b, ta, tb, bias, "none", torch.bfloat16, None, 0.0, plan, add)
    run.mode = mode

    C.set_ws_finish(True)  # opt-in path (off by default: slower, see bindings.cpp)
    try:
        _ws_finish_cases(C, run)
    finally:
        C.set_ws_finish(False)


def _ws_finish_cases(C, run):
    mode = run.mode
    for cfg in range(C.CONV_TILE_CONFIGS):
        for sp in (2, 3, 5, 8):
            plan = (cfg + 16 * sp) | 1024
            C.set_ws_finish(False)
            try:
                want = run(plan)
            finally:
                C.set_ws_finish(True)
            got = run(plan)
            if mode == 2 and sp >= 8:
                torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-4)
            else:
                assert torch.equal(got, want), (cfg, sp)
            assert torch.equal(run(plan), got), (cfg, sp, "rerun")
    # graph replay: the captured launches keep their ticket slices and leave them zeroed
    plan = (2 + 16 * 3) | 1024
    want = run(plan)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run(plan)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = run(plan)
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, want)


def test_gemm_round3_library_plan_entry_falls_back():
    """A round-3 tuning table may still hold library plans (flag 4096); the library plan is gone,
    such an entry runs the heuristic MFMA plan: the result is bit-identical to plan -1's."""
    a, b = bf(512, 768), bf(1024, 768)
    ref = native().gemm(a, b, False, True, None, "none", torch.float32, None, 0.0, -1)
    out = native().gemm(a, b, False, True, None, "none", torch.float32, None, 0.0, 4096)
    assert torch.equal(out, ref)


def test_gemm_identity_asymmetric():
    # A = I with asymmetric B catches transposed C writes (cdna guide §3)
    M = 64
    a = torch.eye(M, device=dev).to(torch.bfloat16)
    b = (torch.arange(M * 128, device=dev).reshape(128, M) % 37).to(torch.bfloat16)  # [N][K]
    out = native().gemm(a, b, False, True, None, "none", torch.float32, None, 0.0)
    assert torch.equal(out, b.float().t())


@pytest.mark.parametrize("C,P", [(64, 37), (256, 16), (2048, 16)])
def test_bn_pipeline(C, P):
    M = 5000
    psum = torch.randn(P, C, device=dev) * 10
    psq = torch.rand(P, C, device=dev) * 100 + 400
    shift = torch.randn(C, device=dev)
    gamma = torch.rand(C, device=dev) + 0.5
    beta = torch.randn(C, device=dev)
    rm, rv = torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5
    rm2, rv2 = rm.clone(), rv.clone()
    # reference first: the native finalize re-zeroes the (replica) slabs it consumed
    ref = _ref.bn_finalize(psum.clone(), psq.clone(), M, shift, gamma, beta, rm2, rv2, 0.1, 1e-5)
    nbt = torch.tensor(7, dtype=torch.int64, device=dev)
    out = native().bn_finalize(psum, psq, M, shift, gamma, beta, rm, rv, 0.1, 1e-5, True, nbt)
    assert int(nbt) == 8
    assert float(psum.abs().max()) == 0.0 and float(psq.abs().max()) == 0.0
    for o, r in zip(out, ref):
        assert rel_err(o, r) < 1e-4
    assert rel_err(rm, rm2) < 1e-5 and rel_err(rv, rv2) < 1e-5
    mean, invstd, scale, bias = ref
    y = bf(M, C)
    r = bf(M, C)
    y2 = bf(M, C)
    for res, rs, rb in [(None, None, None), (r, None, None), (y2, scale * 0.7, bias * 0.3)]:
        z = native().bn_act_fwd(y, scale, bias, True, res, rs, rb)
        zr = _ref.bn_act_fwd(y.float(), scale, bias, True, None if res is None else res.float(), rs, rb)
        assert rel_err(z, zr) < 1e-2
    dz = bf(M, C)
    z = native().bn_act_fwd(y, scale, bias, True, None, None, None)
    sg, sgx, sgx2 = native().bn_act_bwd_reduce(dz, z, y, mean, invstd, True, y2, mean, invstd)
    rg, rgx = _ref.bn_act_bwd_reduce(dz.float(), z, y.float(), mean, invstd, True)
    _, rgx2 = _ref.bn_act_bwd_reduce(dz.float(), z, y2.float(), mean, invstd, True)
    assert rel_err(sg, rg) < 1e-3 and rel_err(sgx, rgx) < 1e-3 and rel_err(sgx2, rgx2) < 1e-3
    dy, dres = native().bn_act_bwd_apply(dz, z, y, mean, invstd, gamma, sg, sgx, M, True, True,
                                         None, None, None, None, None)
    dyr, dresr = _ref.bn_act_bwd_apply(dz.float(), z, y.float(), mean, invstd, gamma, rg, rgx, M,
                                       True, True)
    assert rel_err(dy, dyr) < 2e-2 and rel_err(dres, dresr) < 1e-2
    dy, dy2 = native().bn_act_bwd_apply(dz, z, y, mean, invstd, gamma, sg, sgx, M, True, False,
                                        y2, mean, invstd, gamma * 0.5, sgx2)
    dy2r, _ = _ref.bn_act_bwd_apply(dz.float(), z, y2.float(), mean, invstd, gamma * 0.5, rg, rgx2,
                                    M, True)
    assert rel_err(dy2, dy2r) < 2e-2


def test_maxpool():
    x = bf(2, 17, 16, 64)
    y, idx = native().maxpool_fwd(x, 3, 2, 1)
    yr, _ = _ref.maxpool_fwd(x.float(), 3, 2, 1)
    assert torch.equal(y.float(), yr)
    dy = bf(*y.shape)
    dx = native().maxpool_bwd_impl(dy, idx, list(x.shape), 3, 2, 1)
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    out = torch.nn.functional.max_pool2d(xr, 3, 2, 1)
    out.backward(dy.float().permute(0, 3, 1, 2))
    assert rel_err(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


def test_avgpool():
    x = bf(4, 7, 7, 2048)
    y = native().avgpool_fwd(x)
    assert rel_err(y, _ref.avgpool_fwd(x.float())) < 1e-2
    dy = bf(4, 2048)
    assert rel_err(native().avgpool_bwd(dy, list(x.shape)), _ref.avgpool_bwd(dy.float(), x.shape)) < 1e-2


@pytest.mark.parametrize("V", [1000, 30522])
def test_cross_entropy(V):
    R = 257
    logits = bf(R, V, scale=3.0)
    labels = torch.randint(0, V, (R,), device=dev)
    labels[5] = -100
    for eps in (0.0, 0.1):
        loss, grad = native().cross_entropy_fwd_bwd(logits, labels, eps, -100)
        lr_, gr = _ref.cross_entropy_fwd_bwd(logits.float(), labels, eps, -100)
        assert abs(loss.item() - lr_.item()) / abs(lr_.item()) < 1e-3
        assert rel_err(grad, gr) < 1e-2


@pytest.mark.parametrize("V,valid", [(1000, -1), (30528, 30522), (1001, -1), (10, -1)])
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_cross_entropy_split_fwd_bwd(V, valid, dtype):
    """The training-step split (forward: loss + row log-sum-exps; backward: gradient from the
    logits and a device-side upstream gradient) against the fused kernel and the fp32
    reference — label smoothing, ignored rows, a padded vocabulary (valid columns < V), V % 8
    != 0 (scalar path), fp32 logits, upstream gradient != 1; through mipipe's cross_entropy."""
    from mipipe.ops.functional import cross_entropy
    R = 131
    logits = (torch.randn(R, V, device=dev) * 3).to(dtype)
    labels = torch.randint(0, V if valid < 0 else valid, (R,), device=dev)
    labels[3] = -100
    for eps in (0.0, 0.1):
        loss, work = native().cross_entropy_fwd(logits, labels, eps, -100, valid)
        l0, g0 = native().cross_entropy_fwd_bwd(logits, labels, eps, -100, valid)
        lr_, gr = _ref.cross_entropy_fwd_bwd(logits.float(), labels, eps, -100, valid)
        assert abs(loss.item() - lr_.item()) <= 1e-4 * abs(lr_.item())
        assert abs(loss.item() - l0.item()) <= 1e-5 * abs(l0.item())
        assert int(work[0]) == R - 1
        gout = torch.full((1,), 0.37, device=dev)
        grad = native().cross_entropy_bwd(logits, labels, work, gout, eps, -100, valid)
        assert grad.dtype == dtype
        assert rel_err(grad, gr * 0.37) < (1e-2 if dtype == torch.bfloat16 else 1e-5)
        assert rel_err(grad, g0.float() * 0.37) < (1e-2 if dtype == torch.bfloat16 else 1e-5)
        if valid > 0:
            assert not grad[:, valid:].any()
        assert not grad[3].any()
        x = logits.clone().requires_grad_(True)
        (cross_entropy(x, labels, eps, valid_cols=valid) * 0.37).backward()
        assert torch.equal(x.grad, grad)


def test_sgd_and_adamw():
    n = 4096 * 3
    p = torch.randn(n, device=dev)
    g = torch.randn(n, device=dev)
    m = torch.randn(n, device=dev)
    sh = torch.empty(n, device=dev, dtype=torch.bfloat16)
    p2, m2 = p.clone(), m.clone()
    for first in (True, False):
        native().sgd_step(p, g, m, sh, 0.1, 0.9, 0.0, 1e-4, False, first, 1.0)
        _ref.sgd_step(p2, g, m2, None, 0.1, 0.9, 0.0, 1e-4, False, first)
        assert rel_err(p, p2) < 1e-6 and rel_err(m, m2) < 1e-6
    assert torch.equal(sh, p.to(torch.bfloat16))
    ea, eq = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    ea2, eq2, p3 = ea.clone(), eq.clone(), p.clone()
    for step in (1, 2, 3):
        native().adamw_step(p, g, ea, eq, sh, 1e-3, 0.9, 0.999, 1e-8, 0.01, step, 1.0)
        _ref.adamw_step(p3, g, ea2, eq2, None, 1e-3, 0.9, 0.999, 1e-8, 0.01, step)
    assert rel_err(p, p3) < 1e-5


def test_nchw_to_nhwc_and_synthetic():
    x = torch.randn(3, 3, 11, 13, device=dev)
    y = native().nchw_to_nhwc(x, torch.bfloat16, 8)
    assert y.shape == (3, 11, 13, 8)
    assert torch.equal(y[..., :3], x.permute(0, 2, 3, 1).to(torch.bfloat16))
    assert torch.count_nonzero(y[..., 3:]) == 0
    from mipipe.data.synthetic import synthetic_batch
    idx = torch.arange(10, 74, device=dev)
    xg, lg = native().synthetic_batch(idx, 3, 8, 8, 10, 7, torch.float32)
    xc, lc = synthetic_batch(idx.cpu(), (3, 8, 8), 10, 7)
    assert torch.equal(lg.cpu(), lc)
    assert (xg.cpu() - xc).abs().max() < 1e-3


def test_layernorm_gelu_embedding():
    R, H = 300, 768
    x = bf(R, H)
    res = bf(R, H)
    gma = torch.rand(H, device=dev) + 0.5
    bta = torch.randn(H, device=dev)
    y, mean, rstd, xs = native().layernorm_fwd(x, gma, bta, 1e-12, res)
    yr, mr, rr, xsr = _ref.layernorm_fwd(x.float(), gma, bta, 1e-12, res.float())
    assert rel_err(y, yr) < 1e-2
    dy = bf(R, H)
    dx, dg, db, _ = native().layernorm_bwd(dy, xs, mean, rstd, gma)
    dxr, dgr, dbr = _ref.layernorm_bwd(dy.float(), xs.float(), mean, rstd, gma)
    assert rel_err(dx, dxr) < 2e-2 and rel_err(dg, dgr) < 1e-2 and rel_err(db, dbr) < 1e-2
    g = native().gelu_fwd(x)
    assert rel_err(g, _ref.gelu_fwd(x.float())) < 1e-2
    gb = native().gelu_bwd(dy, x)
    assert rel_err(gb, _ref.gelu_bwd(dy.float(), x.float())) < 1e-2
    idx = torch.randint(0, 50, (R,), device=dev)
    e = native().embedding_bwd(dy, idx, 50)
    assert rel_err(e, _ref.embedding_bwd(dy.float(), idx, 50)) < 1e-3
    cs = native().colsum(dy)
    assert rel_err(cs, dy.float().sum(0)) < 1e-3


@pytest.mark.parametrize("H", [64, 512, 768, 1032, 2048])
@pytest.mark.parametrize("with_res", [False, True])
def test_layernorm_fwd_widths(H, with_res):
    """LayerNorm forward at every chunk count per lane (1..4 x 8 elements, partial last chunk at
    H = 1032), with and without the residual, γ / β given as views off a 16-byte boundary
    (the parameter views of a flat buffer need not be vector-aligned)."""
    R = 37
    x = bf(R, H)
    res = bf(R, H) if with_res else None
    gbuf = torch.rand(H + 1, device=dev) + 0.5
    bbuf = torch.randn(H + 1, device=dev)
    gma, bta = gbuf[1:], bbuf[1:]
    y, mean, rstd, xs = native().layernorm_fwd(x, gma, bta, 1e-5, res)
    # the kernel normalises the bf16-rounded sum (what the backward sees)
    xin = x if res is None else (x.float() + res.float()).to(torch.bfloat16)
    yr, mr, rr, _ = _ref.layernorm_fwd(xin.float(), gma, bta, 1e-5)
    assert rel_err(y, yr) < 1e-2
    assert rel_err(mean, mr) < 1e-3 and rel_err(rstd, rr) < 1e-3
    assert (xs is None) == (res is None)
    if res is not None:
        assert rel_err(xs, x.float() + res.float()) < 1e-2


@pytest.mark.parametrize("mode", [0, 4, 8, 16])
@pytest.mark.parametrize("H", [256, 512, 768, 1024, 1032])
@pytest.mark.parametrize("R", [37, 4100])
def test_layernorm_kernel_modes(mode, H, R):
    """Every LayerNorm kernel family (0: generic 16-B chunks; 4 / 8 / 16: exact-width chunks with
    that many waves per backward block) against the fp32 reference, forward and backward, with
    the fused residual dropout and the producing Linear's bias-gradient sum; row counts that
    leave waves of the last block without rows.  H = 1032 takes the generic kernels in every
    mode."""
    old = native().get_layernorm_mode()
    native().set_layernorm_mode(mode)
    try:
        torch.manual_seed(H + R)
        x, res, dy = bf(R, H), bf(R, H), bf(R, H)
        gbuf = torch.rand(H + 1, device=dev) + 0.5
        gma, bta = gbuf[1:], torch.randn(H, device=dev)
        y, mean, rstd, xs = native().layernorm_fwd(x, gma, bta, 1e-5, res)
        yr, mr, rr, _ = _ref.layernorm_fwd(xs.float(), gma, bta, 1e-5)
        assert rel_err(xs, x.float() + res.float()) < 1e-2
        assert rel_err(y, yr) < 1e-2 and rel_err(mean, mr) < 1e-3 and rel_err(rstd, rr) < 1e-3
        dx, dg, db, _ = native().layernorm_bwd(dy, xs, mean, rstd, gma)
        dxr, dgr, dbr = _ref.layernorm_bwd(dy.float(), xs.float(), mean, rstd, gma)
        assert rel_err(dx, dxr) < 2e-2 and rel_err(dg, dgr) < 1e-3 and rel_err(db, dbr) < 1e-3
        # fused dropout + bias-gradient sum: the dropped branch's gradient and its column sums
        seed = 1234
        ydrop = native().layernorm_fwd(x, gma, bta, 1e-5, res, 0.1, seed)
        x_d = native().dropout_fwd(x, 0.1, seed)
        assert torch.equal(ydrop[3], (x_d.float() + res.float()).to(torch.bfloat16))
        dacc = torch.zeros(H, device=dev)
        gacc, bacc = torch.zeros(H, device=dev), torch.zeros(H, device=dev)
        dx2, _, _, dxd = native().layernorm_bwd(dy, ydrop[3], ydrop[1], ydrop[2], gma, gacc,
                                                bacc, 0.1, seed, None, dacc)
        assert torch.equal(dxd, native().dropout_fwd(dx2, 0.1, seed))
        assert rel_err(dacc, dxd.float().sum(0)) < 1e-3
    finally:
        native().set_layernorm_mode(old)


@pytest.mark.parametrize("M,N,K", [(64, 10, 2048), (30, 100, 512), (64, 16, 27)])
def test_gemm_odd_sizes_padded(M, N, K):
    """Odd sizes (10/100-class heads) go through the zero-padded path of ops.kernels.gemm."""
    from mipipe.ops import kernels as Kx
    x = bf(M, K)
    w = bf(N, K)
    bias = torch.randn(N, device=dev)
    y = Kx.gemm(x, w, False, True, bias, "none", torch.bfloat16)
    assert y.shape == (M, N)
    assert rel_err(y, x.float() @ w.float().t() + bias) < 1e-2
    dy = bf(M, N)
    g = torch.zeros(N, K, device=dev)
    Kx.gemm(dy, x, True, False, None, "none", torch.float32, g, 1.0)
    assert rel_err(g, dy.float().t() @ x.float()) < 2e-3
    dx = Kx.gemm(dy, w, False, False, None, "none", torch.bfloat16)
    assert rel_err(dx, dy.float() @ w.float()) < 1e-2


@pytest.mark.parametrize("case", [(2, 16, 16, 64, 64, 3, 1, 1), (2, 16, 16, 128, 256, 1, 1, 0),
                                  (2, 16, 16, 128, 128, 3, 2, 1), (2, 14, 14, 64, 256, 1, 2, 0)])
def test_conv_dgrad_fused_epilogues(case):
    """dgrad + residual addend + BN-backward reduction epilogue vs the unfused reference."""
    N, H, W, Ci, Co, k, s, p = case
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = bf(N, Ho, Wo, Co)
    w = bf(Co, k, k, Ci, scale=0.1)
    add = bf(N, H, W, Ci)
    y = bf(N, H, W, Ci)
    mean = torch.randn(Ci, device=dev) * 0.1
    invstd = torch.rand(Ci, device=dev) + 0.5
    scale = torch.randn(Ci, device=dev)
    bias = torch.randn(Ci, device=dev) * 0.3
    R = native().STAT_REPLICAS
    rep = torch.zeros(3, R, Ci, device=dev)
    g = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, add, y, mean, invstd, scale, bias, rep)
    dx = _ref.conv_dgrad(dy.float(), w.float(), (N, H, W, Ci), s, p) + add.float()
    mask = (y.float() * scale + bias) > 0
    g_ref = dx * mask
    assert rel_err(g, g_ref) < 2e-2
    xh = (y.float() - mean) * invstd
    gb = g.float()  # stats are of the stored bf16 g
    sg_ref = gb.reshape(-1, Ci).sum(0)
    sgx_ref = (gb * xh).reshape(-1, Ci).sum(0)
    dgam = torch.zeros(Ci, device=dev)
    dbet = torch.ones(Ci, device=dev)
    sg, sgx = native().bn_bwd_collect(rep, Ci, dgam, dbet)
    assert rel_err(sg, sg_ref) < 1e-3 and rel_err(sgx, sgx_ref) < 1e-3
    assert rel_err(dgam, sgx_ref) < 1e-3 and rel_err(dbet - 1, sg_ref) < 1e-3
    assert float(rep.abs().max()) == 0.0  # collect re-zeroes the slab
    only_add = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, add)
    assert rel_err(only_add, dx) < 2e-2


@pytest.mark.parametrize("case", [(2, 16, 16, 64, 64, 3, 1, 1), (2, 14, 14, 64, 256, 1, 2, 0),
                                  (4, 7, 7, 512, 2048, 1, 1, 0)])
def test_bn_collect_rides_in_wgrad(case):
    """The weight-grad launch collects the slab the fused dgrad filled (BnCollect): same Σg /
    Σg·x̂ / dγ / dβ as bn_bwd_collect, slab re-zeroed, weight gradient unchanged."""
    N, H, W, Ci, Co, k, s, p = case
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    dy = bf(N, Ho, Wo, Co)
    w = bf(Co, k, k, Ci, scale=0.1)
    x = bf(N, H, W, Ci)
    y = bf(N, H, W, Ci)
    mean = torch.randn(Ci, device=dev) * 0.1
    invstd = torch.rand(Ci, device=dev) + 0.5
    scale = torch.randn(Ci, device=dev)
    bias = torch.randn(Ci, device=dev) * 0.3
    R = native().STAT_REPLICAS
    reps = [torch.zeros(3, R, Ci, device=dev) for _ in range(2)]
    for rep in reps:
        native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, None, y, mean, invstd, scale, bias, rep)
    dgam, dbet = torch.zeros(Ci, device=dev), torch.ones(Ci, device=dev)
    sg, sgx = native().bn_bwd_collect(reps[0], Ci, dgam, dbet)
    dgam2, dbet2 = torch.zeros(Ci, device=dev), torch.ones(Ci, device=dev)
    out2 = torch.full((2, Ci), float("nan"), device=dev)
    dw = native().conv_wgrad(dy, x, k, k, s, p, col_rep=reps[1], col_out=out2,
                             col_dgamma=dgam2, col_dbeta=dbet2)
    dw_ref = native().conv_wgrad(dy, x, k, k, s, p)
    assert rel_err(dw, dw_ref) < 1e-5
    assert rel_err(out2[0], sg) < 1e-4 and rel_err(out2[1], sgx) < 1e-4
    assert rel_err(dgam2, dgam) < 1e-4 and rel_err(dbet2 - 1, dbet - 1) < 1e-4
    assert float(reps[1].abs().max()) == 0.0
    # without accumulators
    native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, None, y, mean, invstd, scale, bias, reps[1])
    out3 = torch.empty(2, Ci, device=dev)
    native().conv_wgrad(dy, x, k, k, s, p, col_rep=reps[1], col_out=out3)
    assert rel_err(out3[1], sgx) < 1e-3 and float(reps[1].abs().max()) == 0.0


def test_conv_fwd_bias_relu_epilogue():
    N, H, W, Ci, Co = 2, 12, 12, 64, 96
    x = bf(N, H, W, Ci)
    w = bf(Co, 3, 3, Ci, scale=0.1)
    b = torch.randn(Co, device=dev)
    y, _, _ = native().conv_fwd(x, w, 1, 1, None, None, None, b, True)
    ref, _, _ = _ref.conv_fwd(x.float(), w.float(), 1, 1)
    ref = torch.relu(ref + b)
    assert rel_err(y, ref) < 1e-2


def test_stem_superpixel_conv_matches_direct():
    """Packed stem (super-pixels, stride (2,1)) == 7x7/2 pad-3 conv on the image, fwd + wgrad."""
    from mipipe.ops import kernels as Kx
    from mipipe.models.resnet import _StemConv
    N, H, W = 2, 38, 30
    conv = _StemConv(3, 64, 7, stride=2, padding=3, bias=False).cuda()
    x = torch.randn(N, 3, H, W, device=dev)
    xp = conv.pack_input(x, torch.bfloat16)
    Ho, Wo, Hp, Wsp = conv.packed_geometry(H, W)
    assert xp.shape == (N, Hp, Wsp, 8)
    xr = Kx.stem_pack(x.cpu(), torch.float32, 3, Hp, Wsp)
    assert torch.equal(xp.float().cpu(), xr.to(torch.bfloat16).float())
    wk = conv.compute_weight(torch.bfloat16)  # packed by the pack_input launch
    assert torch.equal(wk, conv.compute_weight(torch.bfloat16))  # == the torch-built packing
    # the packed filter gradient accumulates straight into a strided (channels_last) gradient
    conv._ensure_wgrad_map()
    dwp = torch.randn(64, 7, 4, 8, device=dev)
    g0 = torch.randn(64, 3, 7, 7, device=dev).to(memory_format=torch.channels_last)
    g = g0.clone()
    assert conv.weight._mipipe_wgrad_map.accumulate_into(dwp, g)
    assert torch.equal(g, g0 + conv.weight._mipipe_wgrad_map(dwp))
    y, _, _ = native().conv_fwd(xp, wk, 2, 0, None, None, None, None, False, 1)
    ref = torch.nn.functional.conv2d(x.to(torch.bfloat16).float(),
                                     conv.weight.detach().to(torch.bfloat16).float(), stride=2,
                                     padding=3).permute(0, 2, 3, 1)
    assert y.shape == (N, Ho, Wo, 64)
    assert rel_err(y, ref) < 1e-2
    dy = bf(N, Ho, Wo, 64)
    dwk = native().conv_wgrad(dy, xp, 7, 4, 2, 0, None, 1)
    dw = conv.weight._mipipe_wgrad_map(dwk) if hasattr(conv.weight, "_mipipe_wgrad_map") else None
    if dw is None:  # map is installed on first forward
        conv(xp)
        dw = conv.weight._mipipe_wgrad_map(dwk)
    dw_ref = torch.nn.grad.conv2d_weight(x.to(torch.bfloat16).float(), (64, 3, 7, 7),
                                         dy.permute(0, 3, 1, 2).float(), stride=2, padding=3)
    assert rel_err(dw, dw_ref) < 1e-2


TILE_CASES = [
    # N, H, W, Ci, Co, k, s, p  — dense 1x1, gathered 3x3, strided, odd channel counts
    (4, 14, 14, 256, 512, 1, 1, 0),
    (8, 14, 14, 256, 64, 1, 1, 0),  # short-K 1x1 data-grad: epilogue operands primed early
    (4, 15, 13, 64, 192, 3, 1, 1),
    (4, 16, 16, 128, 256, 3, 2, 1),
    (2, 9, 7, 40, 72, 3, 1, 1),
]


SPLIT_CASES = [
    # N, H, W, Ci, Co, k, s, p — small-spatial layers (ResNet-18 32x32 layer 3 / 4 shapes), the
    # dense 1x1, a strided conv (split forward; its data-grad classes are not forward-style) and
    # odd channel counts (unaligned im2col, rows past M, columns past N)
    (16, 2, 2, 256, 256, 3, 1, 1),
    (32, 1, 1, 512, 512, 1, 1, 0),
    (8, 4, 4, 128, 256, 3, 2, 1),
    (3, 7, 5, 40, 72, 3, 1, 1),
]


@pytest.mark.parametrize("splits", [2, 3, 4, 8])
@pytest.mark.parametrize("tile", [0, 2, 8, 1, 9, 11, 14])
@pytest.mark.parametrize("case", SPLIT_CASES)
@DTYPES
def test_conv_split_k_plans(splits, tile, case, dt):
    """Split-K conv plans (plan = tile + 16 x splits): the k-steps run in `splits` slices into an
    fp32 workspace and a finish launch sums the slices in order and runs the regular epilogue —
    forward (+BN statistics, +bias/ReLU) and the forward-style data-grad (+residual addend,
    +BN-backward sums) equal the reference; deterministic mode (statistics as per-tile rows) gives
    bit-identical reruns."""
    f32 = dt == torch.float32
    if f32 and tile not in (0, 2, 8):
        pytest.skip("fp32 runs the 4-wave split-bf16x3 tiles")
    from mipipe.ops import determinism
    N, H, W, Ci, Co, k, s, p = case
    cfg = tile + 16 * splits
    R = (lambda t: t.detach().double().cpu()) if f32 else (lambda t: t.float())
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = rnd(dt, N, H, W, Ci)
    w = rnd(dt, Co, k, k, Ci, scale=1.0 / math.sqrt(Ci * k * k))
    shift = torch.randn(Co, device=dev) * 0.1
    y, ps, pss = native().conv_fwd(x, w, s, p, shift, cfg=cfg)
    yr, psr, pssr = _ref.conv_fwd(R(x), R(w), s, p, R(shift))
    assert rel_err(y, yr) < TOL_OUT[dt]
    # bf16: statistics of the stored (bf16-rounded) outputs over as few as 32 rows
    tol_st = TOL_ACC[dt] if f32 else 5e-3
    assert rel_err(ps.sum(0), psr[0]) < tol_st and rel_err(pss.sum(0), pssr[0]) < tol_st
    bias = torch.randn(Co, device=dev) * 0.1
    yb = native().conv_fwd(x, w, s, p, None, bias=bias, relu=True, cfg=cfg)[0]
    assert rel_err(yb, torch.relu(yr + R(bias))) < TOL_OUT[dt]
    dy = rnd(dt, N, Ho, Wo, Co)
    dxr = _ref.conv_dgrad(R(dy), R(w), (N, H, W, Ci), s, p)
    dx = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, cfg=cfg)
    assert rel_err(dx, dxr) < TOL_OUT[dt]
    yin, add = rnd(dt, N, H, W, Ci), rnd(dt, N, H, W, Ci)
    mean = torch.randn(Ci, device=dev) * 0.1
    invstd = torch.rand(Ci, device=dev) + 0.5
    scale = torch.rand(Ci, device=dev) + 0.5
    bb = torch.randn(Ci, device=dev) * 0.1
    rep = torch.zeros(3, native().STAT_REPLICAS, Ci, device=dev)
    g = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, add, yin, mean, invstd, scale, bb, rep,
                            cfg=cfg)
    sg, sgx = native().bn_bwd_collect(rep, Ci)
    gr = (dxr + R(add)) * ((R(yin) * R(scale) + R(bb)) > 0)
    assert rel_err(g, gr) < TOL_OUT[dt]
    grb = gr if f32 else gr.to(torch.bfloat16).float()
    tol_sum = 1e-4 if f32 else 8e-3
    assert rel_err(sg, grb.reshape(-1, Ci).sum(0)) < tol_sum
    assert rel_err(sgx, (grb * (R(yin) - R(mean)) * R(invstd)).reshape(-1, Ci).sum(0)) < tol_sum
    with determinism.deterministic(True):
        outs = []
        for _ in range(2):
            y1, a1, b1 = native().conv_fwd(x, w, s, p, shift, cfg=cfg)
            rep1 = torch.zeros(3, native().STAT_REPLICAS, Ci, device=dev)
            g1 = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, add, yin, mean, invstd, scale, bb,
                                     rep1, cfg=cfg)
            outs.append((y1, a1, b1, g1, rep1))
        for u, v in zip(*outs):
            assert torch.equal(u, v)
        assert rel_err(outs[0][0], yr) < TOL_OUT[dt]
        assert rel_err(outs[0][1].sum(0), psr[0]) < tol_st


@pytest.mark.parametrize("cfg", list(range(15)))
@pytest.mark.parametrize("case", TILE_CASES)
@DTYPES
def test_conv_every_tile_config(cfg, case, dt):
    """Every tile config of the tuning table (block tile / LDS stages / 4- or 8-wave grid) gives
    the same convolution: fwd (+BN statistics), dgrad (+fused BN-backward epilogue), wgrad
    (heuristic / unsplit / 3-way / 6-way / 12-way split-K).  fp32 (the reference's precision)
    runs tiles 0 / 2 / 8 on the split-bf16x3 loop (other ids resolve to the default tile) and
    is compared with a float64 reference at 1e-4."""
    N, H, W, Ci, Co, k, s, p = case
    f32 = dt == torch.float32
    R = (lambda t: t.detach().double().cpu()) if f32 else (lambda t: t.float())
    Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
    x = rnd(dt, N, H, W, Ci)
    w = rnd(dt, Co, k, k, Ci, scale=1.0 / math.sqrt(Ci * k * k))
    shift = torch.randn(Co, device=dev) * 0.1
    y, ps, pss = native().conv_fwd(x, w, s, p, shift, cfg=cfg)
    yr, psr, pssr = _ref.conv_fwd(R(x), R(w), s, p, R(shift))
    assert y.dtype == dt and rel_err(y, yr) < TOL_OUT[dt]
    assert rel_err(ps.sum(0), psr[0]) < TOL_ACC[dt] and rel_err(pss.sum(0), pssr[0]) < TOL_ACC[dt]
    bias = torch.randn(Co, device=dev) * 0.1
    yb = native().conv_fwd(x, w, s, p, None, bias=bias, relu=True, cfg=cfg)[0]
    assert rel_err(yb, torch.relu(yr + R(bias))) < TOL_OUT[dt]
    dy = rnd(dt, N, Ho, Wo, Co)
    dx = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, cfg=cfg)
    dxr = _ref.conv_dgrad(R(dy), R(w), (N, H, W, Ci), s, p)
    assert dx.dtype == dt and rel_err(dx, dxr) < TOL_OUT[dt]
    # fused epilogue: dx of relu(bn(yin)) with residual addend, BN-backward sums
    yin = rnd(dt, N, H, W, Ci)
    add = rnd(dt, N, H, W, Ci)
    mean = torch.randn(Ci, device=dev) * 0.1
    invstd = torch.rand(Ci, device=dev) + 0.5
    scale = torch.rand(Ci, device=dev) + 0.5
    bias = torch.randn(Ci, device=dev) * 0.1
    rep = torch.zeros(3, native().STAT_REPLICAS, Ci, device=dev)
    g = native().conv_dgrad(dy, w, [N, H, W, Ci], s, p, add, yin, mean, invstd, scale, bias, rep,
                            cfg=cfg)
    sg, sgx = native().bn_bwd_collect(rep, Ci)
    gr = (dxr + R(add)) * ((R(yin) * R(scale) + R(bias)) > 0)
    assert rel_err(g, gr) < TOL_OUT[dt]
    # sums of the stored g: in bf16 the kernel's g and the reference's differ by bf16 rounding
    # of slightly different dx, so the bound is the bf16 sum noise, not fp32's
    grb = gr if f32 else gr.to(torch.bfloat16).float()
    xhat = (R(yin) - R(mean)) * R(invstd)
    tol_sum = 1e-4 if f32 else 8e-3
    assert rel_err(sg, grb.reshape(-1, Ci).sum(0)) < tol_sum
    assert rel_err(sgx, (grb * xhat).reshape(-1, Ci).sum(0)) < tol_sum
    dwr = _ref.conv_wgrad(R(dy), R(x), k, k, s, p)
    # weight-grad plans: heuristic split, unsplit (read-modify-write), 3 / 6 / 12-way split
    for sp in (0, 1, 3, 6, 12):
        dw = native().conv_wgrad(dy, x, k, k, s, p, cfg=cfg + 16 * sp)
        assert rel_err(dw, dwr) < TOL_WGRAD[dt], sp
        acc = torch.ones_like(dw)
        native().conv_wgrad(dy, x, k, k, s, p, acc, cfg=cfg + 16 * sp)
        assert rel_err(R(acc) - 1, dwr) < TOL_WGRAD[dt], sp


def test_tile_benchmark_mode_picks_and_caches():
    C = native()
    C.clear_tune_table()
    C.set_benchmark(True, False, 1)
    try:
        x = bf(8, 14, 14, 256)
        w = bf(256, 3, 3, 256, scale=1 / 48)
        y, _, _ = C.conv_fwd(x, w, 1, 1)
        tab = C.tune_table()
        # a plan: tile id + 16 x split-K count (split plans are candidates for small grids)
        plan = next(iter(tab.values()))
        assert len(tab) == 1 and 0 <= plan % 16 < C.CONV_TILE_CONFIGS and plan // 16 <= 8
        y2, _, _ = C.conv_fwd(x, w, 1, 1)
        assert torch.equal(y, y2) and len(C.tune_table()) == 1
    finally:
        C.set_benchmark(False)
        C.clear_tune_table()


@pytest.mark.parametrize("C", [64, 256])
def test_relu_bitmask_matches_stored_z(C):
    """bn_act_fwd(mask=) writes z > 0 as bits; the fused BN-backward dgrad epilogue reading the
    bits gives exactly what it gives reading z (g and the Σg, Σg·x̂ partials)."""
    N, H, W, Co = 4, 14, 14, 64
    y = bf(N, H, W, C, scale=2.0)
    res = bf(N, H, W, C)
    scale = torch.rand(C, device=dev) + 0.5
    bias = torch.randn(C, device=dev) * 0.1
    mask = torch.empty(N * H * W * C // 8, dtype=torch.uint8, device=dev)
    z = native().bn_act_fwd(y, scale, bias, True, res, None, None, mask)
    bits = (z.reshape(-1, C // 8, 8) > 0).to(torch.int32)
    expect = (bits << torch.arange(8, device=dev, dtype=torch.int32)).sum(-1).to(torch.uint8)
    assert torch.equal(mask, expect.reshape(-1))
    dy = bf(N, H, W, Co)
    w = bf(Co, 1, 1, C, scale=1.0 / math.sqrt(Co))
    add = bf(N, H, W, C)
    mean = torch.randn(C, device=dev) * 0.1
    invstd = torch.rand(C, device=dev) + 0.5
    outs = []
    for kw in (dict(bn_z=z), dict(bn_mask=mask)):
        rep = torch.zeros(3, native().STAT_REPLICAS, C, device=dev)
        g = native().conv_dgrad(dy, w, [N, H, W, C], 1, 0, add, y, mean, invstd, scale, bias, rep,
                                **kw)
        outs.append((g, *native().bn_bwd_collect(rep, C)))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-5)
    assert torch.allclose(outs[0][2], outs[1][2], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("shape", [(4, 32, 32, 64), (2, 17, 15, 64), (3, 12, 12, 128)])
@pytest.mark.parametrize("det", [0, 1])
def test_pool_bn_fused_matches_unfused(shape, det):
    """Stem fusion: maxpool(relu(bn(y))) in one kernel + gather backward == the unfused
    BN-apply -> max-pool -> max-pool backward -> BN reduce -> BN apply chain."""
    from mipipe.ops import kernels as Kx
    from mipipe.ops import determinism
    N, H, W, C = shape
    y = bf(N, H, W, C)
    scale = torch.randn(C, device=dev)
    bias = torch.randn(C, device=dev) * 0.5
    mean = torch.randn(C, device=dev) * 0.1
    invstd = torch.rand(C, device=dev) + 0.5
    gamma = torch.randn(C, device=dev)
    count = N * H * W
    R = native().STAT_REPLICAS
    old = determinism.deterministic_enabled()
    determinism.set_deterministic(bool(det))
    try:
        out, idx = Kx.pool_bn_fwd(y, scale, bias, 3, 2, 1)
        z = Kx.bn_act_fwd(y, scale, bias, True)
        out2, idx2 = Kx.maxpool_fwd(z, 3, 2, 1)
        assert torch.equal(out, out2) and torch.equal(idx, idx2)
        dp = bf(*out.shape)
        rep = torch.zeros(3, R, C, device=dev)
        dg, db = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        dy, sg, sgx = Kx.pool_bn_bwd(dp, idx, out, y, mean, invstd, gamma, rep, count, 3, 2, 1,
                                     acc=(dg, db))
        assert float(rep.abs().max()) == 0.0
        dz = Kx.maxpool_bwd(dp, idx2, z.shape, 3, 2, 1)
        rep2 = torch.zeros(3, R, C, device=dev)
        sg2, sgx2, _ = Kx.bn_act_bwd_reduce(dz, z, y, mean, invstd, True, rep=rep2)
        dy2, _ = Kx.bn_act_bwd_apply(dz, z, y, mean, invstd, gamma, sg2, sgx2, count, True)
        assert rel_err(sg, sg2) < 1e-4 and rel_err(sgx, sgx2) < 1e-4
        assert rel_err(dg, sgx2) < 1e-4 and rel_err(db - 1, sg2) < 1e-4
        assert rel_err(dy, dy2) < 1e-2
    finally:
        determinism.set_deterministic(old)


@pytest.mark.parametrize("case", [(2, 16, 16, 256, 64), (4, 7, 7, 2048, 512), (8, 28, 28, 512, 128)])
@pytest.mark.parametrize("det", [0, 1])
def test_conv_dgrad_two_branch_bn_fusion(case, det):
    """Downsample-block output relu(bn(y) + bn2(y2)) consumed by a 1x1 conv: its dgrad epilogue
    masks g with the stored ReLU bits, adds the identity gradient and reduces Σg, Σg·x̂, Σg·x̂₂;
    the weight-grad launch collects all three (dγ/dβ, dγ₂/dβ₂ accumulated)."""
    from mipipe.ops import determinism
    N, H, W, Ci, Co = case
    dy = bf(N, H, W, Co)
    w = bf(Co, 1, 1, Ci, scale=0.05)
    x = bf(N, H, W, Ci)
    add = bf(N, H, W, Ci)
    y, y2 = bf(N, H, W, Ci), bf(N, H, W, Ci)
    mean, mean2 = torch.randn(Ci, device=dev) * 0.1, torch.randn(Ci, device=dev) * 0.1
    invstd, invstd2 = torch.rand(Ci, device=dev) + 0.5, torch.rand(Ci, device=dev) + 0.5
    scale, bias = torch.randn(Ci, device=dev), torch.randn(Ci, device=dev) * 0.3
    z = bf(N, H, W, Ci)  # any tensor: the mask is its sign
    bits = torch.empty(z.numel() // 8, dtype=torch.uint8, device=dev)
    zz = native().bn_act_fwd(z, torch.ones(Ci, device=dev), torch.zeros(Ci, device=dev), True,
                             None, None, None, bits)
    R = native().STAT_REPLICAS
    rep = torch.zeros(3, R, Ci, device=dev)
    old = determinism.deterministic_enabled()
    determinism.set_deterministic(bool(det))
    try:
        g = native().conv_dgrad(dy, w, [N, H, W, Ci], 1, 0, add, y, mean, invstd, scale, bias,
                                rep, None, bn_mask=bits, bn_y2=y2, bn_mean2=mean2,
                                bn_invstd2=invstd2)
        out3 = torch.empty(3, Ci, device=dev)
        dg, db, dg2, db2 = (torch.zeros(Ci, device=dev) for _ in range(4))
        native().conv_wgrad(dy, x, 1, 1, 1, 0, col_rep=rep, col_out=out3, col_dgamma=dg,
                            col_dbeta=db, col_two=True, col_dgamma2=dg2, col_dbeta2=db2)
    finally:
        determinism.set_deterministic(old)
    dx = _ref.conv_dgrad(dy.float(), w.float(), (N, H, W, Ci), 1, 0) + add.float()
    g_ref = dx * (zz.float() > 0)
    assert rel_err(g, g_ref) < 2e-2
    gb = g.float().reshape(-1, Ci)
    sg = gb.sum(0)
    sgx = (gb * ((y.float() - mean) * invstd).reshape(-1, Ci)).sum(0)
    sgx2 = (gb * ((y2.float() - mean2) * invstd2).reshape(-1, Ci)).sum(0)
    assert rel_err(out3[0], sg) < 1e-3 and rel_err(out3[1], sgx) < 1e-3
    assert rel_err(out3[2], sgx2) < 1e-3
    assert rel_err(dg, sgx) < 1e-3 and rel_err(db, sg) < 1e-3
    assert rel_err(dg2, sgx2) < 1e-3 and rel_err(db2, sg) < 1e-3
    assert float(rep.abs().max()) == 0.0


@pytest.mark.parametrize("rows,H,n", [(30528, 768, 4096), (512, 768, 4096), (2, 768, 4096),
                                      (50, 64, 300), (1000, 1032, 777)])
def test_embedding_bwd_ordered(rows, H, n):
    """Ordered (deterministic) embedding backward: stable sort of the ids and one writer per
    table row (or per-block tables summed in order for <= 8 rows) — equals the fp32 reference,
    is bit-identical run to run, accumulates into `out` and applies `scale`."""
    dy = bf(n, H)
    idx = torch.randint(0, rows, (n,), device=dev)
    idx[: n // 4] = idx[0]  # one long run of equal ids (a frequent token)
    ref = _ref.embedding_bwd(dy.float(), idx, rows)
    a = native().embedding_bwd(dy, idx, rows, None, True)
    b = native().embedding_bwd(dy, idx, rows, None, True)
    assert torch.equal(a, b)
    assert rel_err(a, ref) < 1e-5
    acc = torch.randn(rows, H, device=dev)
    acc0 = acc.clone()
    native().embedding_bwd(dy, idx, rows, acc, True, 0.125)
    assert rel_err(acc - acc0, 0.125 * ref) < 1e-4


@pytest.mark.parametrize("rows,H,n", [(2, 768, 4096), (8, 64, 777), (1, 1032, 300), (5, 2048, 129)])
def test_embedding_bwd_tiny_tables(rows, H, n):
    """Tables of <= 8 rows (token types): register accumulation per 8-column chunk and token
    stream, streams added in order — default (atomics into out) and ordered paths against the
    fp32 reference; the ordered one bit-identical run to run."""
    dy = bf(n, H)
    idx = torch.randint(0, rows, (n,), device=dev)
    ref = _ref.embedding_bwd(dy.float(), idx, rows)
    assert rel_err(native().embedding_bwd(dy, idx, rows), ref) < 1e-5
    a = native().embedding_bwd(dy, idx, rows, None, True)
    b = native().embedding_bwd(dy, idx, rows, None, True)
    assert torch.equal(a, b) and rel_err(a, ref) < 1e-5


@pytest.mark.parametrize("n,pad_frac,run_frac", [(32768, 0.0, 0.3), (32768, 0.25, 0.0),
                                                  (4096, 0.1, 0.9), (130, 0.0, 1.0),
                                                  (64, 0.5, 0.0), (65, 0.0, 1.0)])
def test_embedding_bwd_presorted_chunked(n, pad_frac, run_frac):
    """The DDP exchange's scatter: ids sorted ahead (presorted), padding rows with id -1
    (skipped), and one id repeated over a long run spanning many 64-entry chunks (a [PAD]
    token) — summed in parallel per chunk, then the chunk partials in order.  Equals the
    float64 reference, bit-identical run to run and to the self-sorting ordered path."""
    rows, H = 30528, 768
    dy = bf(n, H)
    idx = torch.randint(0, rows, (n,), device=dev)
    idx[: int(n * run_frac)] = 3
    npad = int(n * pad_frac)
    if npad:
        idx[-npad:] = -1
        dy[-npad:] = float("nan")  # must never be read
    sid, perm = torch.sort(idx, stable=True)
    keep = idx >= 0
    ref = torch.zeros(rows, H, dtype=torch.float64, device=dev)
    ref.index_add_(0, idx[keep], dy[keep].double())
    a = torch.zeros(rows, H, device=dev)
    native().embedding_bwd(dy, idx, rows, a, True, 0.5, sid, perm)
    b = torch.zeros(rows, H, device=dev)
    native().embedding_bwd(dy, idx, rows, b, True, 0.5, sid, perm)
    assert torch.equal(a, b)
    assert not torch.isnan(a).any()
    assert rel_err(a, 0.5 * ref) < 1e-6
    if not npad:
        c = torch.zeros(rows, H, device=dev)
        native().embedding_bwd(dy, idx, rows, c, True, 0.5)
        assert torch.equal(a, c)


@pytest.mark.parametrize("M,N,K", [(4096, 3072, 768), (640, 768, 768), (200, 136, 72)])
def test_gemm_gelu_epilogue_matches_gemm_then_gelu(M, N, K):
    """The GELU Linear forward in one GEMM (pre-activation to aux, GELU to the output) ==
    the plain bias GEMM followed by the gelu_fwd kernel, bit for bit, for every tile config."""
    from mipipe.ops import kernels as Kk
    C = native()
    x, w = bf(M, K), bf(N, K, scale=0.05)
    bias = torch.randn(N, device=dev)
    for cfg in range(C.CONV_TILE_CONFIGS):
        h0 = C.gemm(x, w, False, True, bias, "none", torch.bfloat16, None, 0.0, cfg)
        y0 = Kk.gelu_fwd(h0)
        y1, h1 = C.gemm_gelu(x, w, bias, cfg)
        assert torch.equal(h0, h1), cfg
        assert torch.equal(y0, y1), cfg
    ref = torch.nn.functional.gelu(x.float() @ w.float().t() + bias)
    assert rel_err(y1, ref) < 1e-2
