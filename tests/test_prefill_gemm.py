"""Hand-written CDNA4 prefill GEMM (ops/csrc/prefill_gemm.hip) vs a plain PyTorch fp32
reference of the same op: plain, residual-add (in place) and SiLU-mul (w = [gate; up])
epilogues, ragged M (row clamping at the last tile), K not a multiple of the 4-phase ring."""
import pytest
import torch

from agentic_traffic_testing_amd import ops


def _ref(x, w, mode, res=None):
    y = x.float() @ w.float().t()
    if mode == ops.GEMM_SILU:
        n = w.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    if mode == ops.GEMM_RESADD:
        y = y + res.float()
    return y


def _check(got, exp, k):
    # bf16 output rounding (2^-8 relative) + fp32 accumulation-order noise
    err = (got.float() - exp).abs()
    tol = 2e-2 * exp.abs() + 2e-3 * k ** 0.5
    assert bool((err <= tol).all()), f"max err {err.max().item():.4g}"


def test_prefill_gemm_cpu_reference_path():
    torch.manual_seed(0)
    x = torch.randn(5, 64, dtype=torch.bfloat16)
    w = torch.randn(512, 64, dtype=torch.bfloat16) / 8
    assert ops.prefill_gemm_ok(x, w) and ops.prefill_gemm_ok(x, w, ops.GEMM_SILU)
    assert not ops.prefill_gemm_ok(x, w[:300])
    _check(ops.prefill_gemm(x, w), _ref(x, w, ops.GEMM_PLAIN), 64)
    _check(ops.prefill_gemm(x, w, ops.GEMM_SILU), _ref(x, w, ops.GEMM_SILU), 64)
    r = torch.randn(5, 512, dtype=torch.bfloat16)
    exp = _ref(x, w, ops.GEMM_RESADD, r)
    assert ops.prefill_gemm(x, w, ops.GEMM_RESADD, residual=r) is r
    _check(r, exp, 64)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("mnk", [(1, 256, 32), (77, 512, 96), (256, 256, 256),
                                 (300, 768, 4096), (1029, 1024, 1056), (2600, 512, 4096)])
def test_prefill_gemm_vs_fp32(mode, mnk):
    assert ops.native_available(), ops._load_error
    M, N, K = mnk
    torch.manual_seed(M + N + K + mode)
    dev = "cuda"
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    rows = 2 * N if mode == ops.GEMM_SILU else N
    w = (torch.randn(rows, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    if mode == ops.GEMM_RESADD:
        r = torch.randn(M, N, device=dev).to(torch.bfloat16)
        exp = _ref(x, w, mode, r)
        got = ops.prefill_gemm(x, w, mode, residual=r)
        assert got is r
    else:
        exp = _ref(x, w, mode)
        got = ops.prefill_gemm(x, w, mode)
    torch.cuda.synchronize()
    assert got.shape == (M, N)
    _check(got, exp, K)


@pytest.mark.gpu
def test_prefill_gemm_strided_rows_and_asymmetric_operands():
    """A with a row stride (a view into a wider buffer) and an asymmetric W: catches a
    transposed C/D map or a wrong swizzle on either side (guide §5 'Common mistakes' 3)."""
    assert ops.native_available(), ops._load_error
    torch.manual_seed(7)
    M, N, K = 333, 512, 1024
    big = torch.randn(M, K + 64, device="cuda").to(torch.bfloat16)
    x = big[:, 32:32 + K]
    w = (torch.arange(N * K, device="cuda").reshape(N, K) % 97 - 48).to(torch.bfloat16) / 64
    _check(ops.prefill_gemm(x, w), _ref(x, w, ops.GEMM_PLAIN), K)
    eye = torch.eye(K, device="cuda", dtype=torch.bfloat16)[:256]
    got = ops.prefill_gemm(x, eye)
    assert torch.equal(got, x[:, :256])


def _q8(t):
    """Row-wise e4m3fn quantisation: (uint8 codes, fp32 scales [rows, 1])."""
    s = (t.float().abs().amax(dim=1, keepdim=True) / 448.0).clamp_min(1e-12)
    q = (t.float() / s).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    return q, s


def _ref8(xq, xs, wq, ws, mode, res=None):
    x = xq.view(torch.float8_e4m3fn).float() * xs.reshape(-1, 1)
    w = wq.view(torch.float8_e4m3fn).float() * ws.reshape(-1, 1)
    y = x @ w.t()
    if mode == ops.GEMM_SILU:
        n = w.shape[0] // 2
        y = torch.nn.functional.silu(y[:, :n]) * y[:, n:]
    if mode == ops.GEMM_RESADD:
        y = y + res.float()
    return y


def test_prefill_gemm_fp8_cpu_reference_path():
    torch.manual_seed(3)
    xq, xs = _q8(torch.randn(7, 128))
    wq, ws = _q8(torch.randn(256, 128))
    assert ops.prefill_gemm_ok(xq, wq)
    _check(ops.prefill_gemm(xq, wq, xs=xs, ws=ws), _ref8(xq, xs, wq, ws, 0), 128)
    with pytest.raises(ValueError):
        ops.prefill_gemm(xq, wq)


@pytest.mark.gpu
def test_prefill_gemm_fp8_exact_integer_layout():
    """Small integers are exact in e4m3 and their products sum exactly in fp32: any error
    in the 32x32x64 f8f6f4 operand or C/D lane maps, or in the LDS swizzle, shows up as a
    mismatch (guide: 'check the map with exact integer data')."""
    assert ops.native_available(), ops._load_error
    M, N, K = 300, 512, 256
    g = torch.Generator().manual_seed(11)
    xi = torch.randint(-3, 4, (M, K), generator=g).float()
    wi = torch.randint(-3, 4, (N, K), generator=g).float()
    wi[:, :64] += torch.arange(N).reshape(-1, 1) % 5  # asymmetric W
    xq = xi.to(torch.float8_e4m3fn).view(torch.uint8).cuda()
    wq = wi.to(torch.float8_e4m3fn).view(torch.uint8).cuda()
    ones_m = torch.ones(M, 1, device="cuda")
    ones_n = torch.ones(N, device="cuda")
    got = ops.prefill_gemm(xq, wq, xs=ones_m, ws=ones_n).float().cpu()
    exp = (xi @ wi.t()).to(torch.bfloat16).float()
    assert torch.equal(got, exp), f"{(got != exp).sum().item()} mismatches"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("mnk", [(1, 256, 64), (77, 512, 192), (300, 768, 4096),
                                 (1029, 1024, 1088), (2600, 512, 4096)])
def test_prefill_gemm_fp8_vs_fp32(mode, mnk):
    assert ops.native_available(), ops._load_error
    M, N, K = mnk
    torch.manual_seed(M + N + K + 10 * mode)
    rows = 2 * N if mode == ops.GEMM_SILU else N
    xq, xs = _q8(torch.randn(M, K, device="cuda"))
    wq, ws = _q8(torch.randn(rows, K, device="cuda") / K ** 0.5)
    ws = ws.reshape(-1).contiguous()
    if mode == ops.GEMM_RESADD:
        r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        exp = _ref8(xq, xs, wq, ws, mode, r)
        got = ops.prefill_gemm(xq, wq, mode, residual=r, xs=xs, ws=ws)
    else:
        exp = _ref8(xq, xs, wq, ws, mode)
        got = ops.prefill_gemm(xq, wq, mode, xs=xs, ws=ws)
    torch.cuda.synchronize()
    assert got.shape == (M, N)
    _check(got, exp, K)
    assert ops.prefill_gemm_error() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("sched", ["hybrid", "streamk", "dp", "splitk"])
@pytest.mark.parametrize("bm", [64, 128, 256])
@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("mnk", [(73, 1024, 4096), (382, 768, 2048), (700, 512, 1024)])
def test_prefill_gemm_tiles_schedules_vs_fp32(sched, bm, mode, mnk):
    """Every tile height (64 / 128 / 256 rows) under every schedule, chosen per call: the
    planning-call (73 rows) and fan-out-burst (382 rows) shapes, ragged M in every tile."""
    assert ops.native_available(), ops._load_error
    M, N, K = mnk
    torch.manual_seed(M + N + K + mode + bm)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    rows = 2 * N if mode == ops.GEMM_SILU else N
    w = (torch.randn(rows, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    kw = dict(schedule=sched, bm=bm)
    if mode == ops.GEMM_RESADD:
        r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        exp = _ref(x, w, mode, r)
        got = ops.prefill_gemm(x, w, mode, residual=r, **kw)
    else:
        exp = _ref(x, w, mode)
        got = ops.prefill_gemm(x, w, mode, **kw)
        # deterministic: partials are summed in a fixed order whoever finishes last
        assert torch.equal(ops.prefill_gemm(x, w, mode, **kw), got)
    torch.cuda.synchronize()
    _check(got, exp, K)
    assert ops.prefill_gemm_error() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("bm", [64, 128, 256])
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_prefill_gemm_fp8_tiles_vs_fp32(bm, mode):
    assert ops.native_available(), ops._load_error
    M, N, K = 382, 1024, 4096
    torch.manual_seed(5 + mode + bm)
    rows = 2 * N if mode == ops.GEMM_SILU else N
    xq, xs = _q8(torch.randn(M, K, device="cuda"))
    wq, ws = _q8(torch.randn(rows, K, device="cuda") / K ** 0.5)
    ws = ws.reshape(-1).contiguous()
    for sched in ("hybrid", "splitk"):
        if mode == ops.GEMM_RESADD:
            r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            exp = _ref8(xq, xs, wq, ws, mode, r)
            got = ops.prefill_gemm(xq, wq, mode, residual=r, xs=xs, ws=ws, schedule=sched, bm=bm)
        else:
            exp = _ref8(xq, xs, wq, ws, mode)
            got = ops.prefill_gemm(xq, wq, mode, xs=xs, ws=ws, schedule=sched, bm=bm)
        torch.cuda.synchronize()
        _check(got, exp, K)
    assert ops.prefill_gemm_error() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("sched", ["streamk", "splitk"])
@pytest.mark.parametrize("mode", [0, 2])
def test_prefill_gemm_timed_out_wait_recomputes(sched, mode):
    """A cross-workgroup wait that gives up (forced: ablate=4 makes every wait time out at
    once) recomputes the tile over the whole K range: the output stays exact and the error
    word says so (bit 4), instead of reading partials nobody wrote."""
    assert ops.native_available(), ops._load_error
    M, N, K = 300, 1024, 4096
    torch.manual_seed(13 + mode)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    rows = 2 * N if mode == ops.GEMM_SILU else N
    w = (torch.randn(rows, K, device="cuda") / K ** 0.5).to(torch.bfloat16)
    exp = _ref(x, w, mode)
    ops.prefill_gemm_config("hybrid", ablate=4)
    try:
        got = ops.prefill_gemm(x, w, mode, schedule=sched, bm=128)
        torch.cuda.synchronize()
    finally:
        ops.prefill_gemm_config("hybrid")
    try:
        _check(got, exp, K)
        assert ops.prefill_gemm_error() & 4
        # the protocol state is re-armed: a normal call afterwards is exact
        ops.prefill_gemm_error_reset()
        got2 = ops.prefill_gemm(x, w, mode, schedule=sched, bm=128)
        torch.cuda.synchronize()
        _check(got2, exp, K)
        assert ops.prefill_gemm_error() == 0  # and times out nowhere
    finally:
        ops.prefill_gemm_error_reset()  # later tests assert a clean word


def test_prefill_gemm_per_call_schedule_keeps_process_config(monkeypatch):
    """schedule= / bm= travel with the call; the process-wide configuration is never touched
    (the old override reset group_m / ablate and left 'splitk' behind)."""
    calls = []

    class Fake:
        def prefill_gemm(self, *a):
            calls.append(("gemm",) + a[-2:])

        def prefill_gemm_config(self, *a):
            calls.append(("config",) + a)

    monkeypatch.setattr(ops, "_native", lambda: Fake())
    before = ops._PG_SCHEDULE
    x = torch.zeros(4, 64, dtype=torch.bfloat16, device="meta")
    w = torch.zeros(256, 64, dtype=torch.bfloat16, device="meta")
    monkeypatch.setattr(torch.Tensor, "is_cuda", property(lambda self: True))
    ops.prefill_gemm(x, w, out=torch.zeros(4, 256, dtype=torch.bfloat16, device="meta"),
                     schedule="splitk", bm=128)
    ops.prefill_gemm(x, w, out=torch.zeros(4, 256, dtype=torch.bfloat16, device="meta"))
    assert calls == [("gemm", 3, 128), ("gemm", -1, 0)]
    assert ops._PG_SCHEDULE == before
