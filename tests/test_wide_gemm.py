"""Wide small-M GEMM (ops/csrc/wide.hip): 12-128 rows over pre-shuffled 16-bit weights with
the decode GEMVs' fused epilogues, against the fp32 PyTorch reference (ops/reference.py).
Every epilogue (plain, residual add, RMSNorm-folded QKV + RoPE + paged K/V write, RMSNorm-
folded gate_up + SiLU-mul, LM head + sampler keys), ragged M from 12 to 128, and every
(waves, K split) plan the library can pick - split-K slices combined in slice order
(bitwise deterministic), arrival counters re-armed."""
import math

import pytest
import torch

from agentic_traffic_testing_amd import ops
from agentic_traffic_testing_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
PLANS = [(0, 0), (4, 1), (8, 1), (6, 3), (7, 2), (8, 8), (4, 5)]


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert ops.native_available(), ops._load_error
    ops.ensure_splitk_workspace("cuda")


def close(a, b, atol, rtol=0.0):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    assert bool((err <= tol).all()), f"max err {err.max().item():.4g}"


def _norm_fits(waves, m):
    """Plans built with the RMSNorm fold (wide.h norm_fits): 6 / 7 waves spill at 113-128
    rows, 6 waves at 97-112."""
    mt = (m + 15) // 16
    return not ((mt == 8 and waves in (6, 7)) or (mt == 7 and waves == 6))


def _norm_ref(x, eps=1e-5):
    return ref.rms_norm(x, torch.ones(x.shape[1], dtype=x.dtype, device=x.device), eps)


@pytest.mark.parametrize("plan", PLANS)
@pytest.mark.parametrize("m,n,k", [(33, 1024, 4096), (85, 4096, 4096), (128, 512, 14336),
                                   (47, 6144, 1024), (96, 2048, 2048), (75, 4096, 4096),
                                   (110, 2048, 2048), (17, 4096, 4096), (24, 2048, 14336)])
def test_wide_linear_plain_and_residual(plan, m, n, k):
    torch.manual_seed(41)
    dt = torch.bfloat16
    x = torch.randn(m, k, dtype=dt, device="cuda")
    w = torch.randn(n, k, dtype=dt, device="cuda") * 0.02
    wp = ops.preshuffle(w)
    exp = x.float() @ w.float().t()
    assert ops.skinny_ok(x, wp, preshuffled=True)
    for _ in range(2):  # counters re-arm
        ops.set_wide_plan(*plan)
        got = ops.linear(x, wp, preshuffled=True)
        close(got, exp, 2e-2 * math.sqrt(k / 4096), 1e-2)
        r = torch.randn(m, n, dtype=dt, device="cuda")
        exp_r = exp.to(dt).float() + r.float()
        ops.set_wide_plan(*plan)
        out = ops.linear(x, wp, residual=r, preshuffled=True)
        assert out.data_ptr() == r.data_ptr()
        close(r, exp_r, 3e-2 * math.sqrt(k / 4096), 1e-2)
    ws, counters = ops._SPLITK_WS[torch.cuda.current_device()]
    assert bool((counters == 0).all())
    ops.set_wide_plan(*plan)
    a = ops.linear(x, wp, preshuffled=True)
    ops.set_wide_plan(*plan)
    b = ops.linear(x, wp, preshuffled=True)
    assert torch.equal(a, b)  # slice-ordered combine: run-to-run bit-identical


@pytest.mark.parametrize("plan", [(0, 0), (6, 4), (8, 1), (4, 3)])
@pytest.mark.parametrize("m", [20, 33, 75, 85, 100, 128])
@pytest.mark.parametrize("hq,hkv,H", [(32, 8, 4096), (8, 1, 8192)])
def test_wide_qkv_rope(plan, m, hq, hkv, H):
    if not _norm_fits(plan[0], m):
        pytest.skip("this wave count x row count with the norm fold is not built (VGPR spill)")
    torch.manual_seed(42)
    dt, bs, nb = torch.bfloat16, 16, 64
    x = torch.randn(m, H, dtype=dt, device="cuda") * 2
    w = torch.randn((hq + 2 * hkv) * 128, H, dtype=dt, device="cuda") * 0.02
    pos = torch.randint(0, 4000, (m,), dtype=torch.int32, device="cuda")
    slots = torch.randperm(nb * bs, device="cuda")[:m].to(torch.int32)
    slots[1] = -1  # a padding row writes no K/V
    cs = ref.rope_cos_sin(128, 8192, 500000.0, None, device="cuda")
    k1 = torch.randn(nb, hkv, bs, 128, dtype=dt, device="cuda")
    v1 = torch.randn(nb, hkv, 128, bs, dtype=dt, device="cuda")
    k2, v2 = k1.clone(), v1.clone()
    q_exp = ref.rope_cache(torch.nn.functional.linear(_norm_ref(x), w), pos, slots, cs, k1, v1,
                           hq, hkv, 128)
    ops.set_wide_plan(*plan)
    q_got = ops.decode_qkv_rope(x, ops.preshuffle(w, "qkv"), 1e-5, pos, slots, cs, k2, v2, hq,
                                hkv, preshuffled=True)
    close(q_got, q_exp, 3e-2, 2e-2)
    close(k2, k1, 3e-2, 2e-2)
    close(v2, v1, 3e-2, 2e-2)


@pytest.mark.parametrize("plan", [(0, 0), (7, 1), (8, 2), (4, 4)])
@pytest.mark.parametrize("m", [12, 16, 27, 40, 75, 85, 100, 128])
@pytest.mark.parametrize("inter,k", [(14336, 4096), (1792, 8192)])
def test_wide_gate_up_silu(plan, m, inter, k):
    if not _norm_fits(plan[0], m):
        pytest.skip("this wave count x row count with the norm fold is not built (VGPR spill)")
    torch.manual_seed(43)
    dt = torch.bfloat16
    x = torch.randn(m, k, dtype=dt, device="cuda")
    w = torch.randn(2 * inter, k, dtype=dt, device="cuda") * 0.02
    exp = ref.silu_and_mul(torch.nn.functional.linear(_norm_ref(x), w))
    ops.set_wide_plan(*plan)
    got = ops.decode_gate_up_silu(x, ops.preshuffle(w, "silu"), 1e-5, preshuffled=True)
    close(got, exp, 4e-2, 4e-2)


@pytest.mark.parametrize("m", [40, 100])
def test_wide_lm_head_sample(m):
    torch.manual_seed(44)
    dt, V, H = torch.bfloat16, 32768, 1024
    x = torch.randn(m, H, dtype=dt, device="cuda")
    w = torch.randn(V, H, dtype=dt, device="cuda") * 0.05
    keys = torch.full((m * V // 16,), -1, dtype=torch.int64, device="cuda")
    temp = torch.zeros(m, device="cuda")
    seeds = torch.arange(m, dtype=torch.int64, device="cuda")
    steps = torch.zeros(m, dtype=torch.int64, device="cuda")
    logits = torch.nn.functional.linear(_norm_ref(x), w).float()
    got = ops.decode_lm_head_sample(x, ops.preshuffle(w), 1e-5, temp, seeds, steps, keys,
                                    preshuffled=True)
    top2 = torch.topk(logits, 2, dim=-1)
    for r in range(m):
        g = int(got[r])
        assert g == int(top2.indices[r, 0]) or float(top2.values[r, 0] - logits[r, g]) < 0.05
    # sampled rows: the same keys as the 16-row-tile kernel on the first 32 rows (identical
    # per-tile math and noise), so the tokens agree
    temp.fill_(0.8)
    a = ops.decode_lm_head_sample(x, ops.preshuffle(w), 1e-5, temp, seeds, steps, keys,
                                  preshuffled=True).clone()
    b = ops.decode_lm_head_sample(x[:32].contiguous(), ops.preshuffle(w), 1e-5, temp[:32],
                                  seeds[:32], steps[:32], keys, preshuffled=True)
    assert (a[:32] == b).float().mean() >= 0.9  # bf16 logit near-ties may flip a draw


def test_wide_matches_skinny_at_the_seam():
    """32 rows (16-row-tile GEMV) and 33 rows (wide kernel): the first 32 output rows agree
    to bf16 rounding - the seam between the two kernels is invisible to the engine."""
    torch.manual_seed(45)
    dt = torch.bfloat16
    x = torch.randn(33, 4096, dtype=dt, device="cuda")
    w = (torch.randn(4096, 4096, dtype=dt, device="cuda") * 0.02)
    wp = ops.preshuffle(w)
    a = ops.linear(x[:32].contiguous(), wp, preshuffled=True)
    b = ops.linear(x, wp, preshuffled=True)
    close(b[:32], a, 2e-2, 1e-2)


# ---- fp8 weights (W8 builds: e4m3fn weight-only quantisation, per-row scales) ----------------
W8_PLANS = [(0, 0), (4, 1), (8, 1), (8, 3), (4, 5)]


def _fp8(w, rowmap="plain"):
    """(pre-shuffled fp8 bytes, row scales, the dequantised fp32 weight the oracle uses)."""
    q, s = ops.quantize_fp8(w)
    deq = q.view(torch.float8_e4m3fn).float() * s[:, None]
    return ops.preshuffle_fp8(q, rowmap), s, deq


@pytest.mark.parametrize("plan", W8_PLANS)
@pytest.mark.parametrize("m,n,k", [(33, 1024, 4096), (85, 4096, 4096), (128, 512, 14336),
                                   (47, 6144, 1024), (100, 2048, 2048)])
def test_wide_fp8_linear_plain_and_residual(plan, m, n, k):
    """33-128 rows over fp8 weights: the wide kernel's W8 builds (weights converted to bf16
    MFMA operands in registers, the row scale on the finished accumulators) against the fp32
    product with the dequantised weights; split-K plans deterministic."""
    torch.manual_seed(46)
    dt = torch.bfloat16
    x = torch.randn(m, k, dtype=dt, device="cuda")
    wq, s, deq = _fp8(torch.randn(n, k, dtype=dt, device="cuda") * 0.02)
    exp = x.float() @ deq.t()
    assert ops.skinny_ok(x, wq, preshuffled=True, fp8=True)
    ops.set_wide_plan(*plan)
    got = ops.linear(x, wq, w_scale=s)
    close(got, exp, 2e-2 * math.sqrt(k / 4096), 1e-2)
    r = torch.randn(m, n, dtype=dt, device="cuda")
    exp_r = exp.to(dt).float() + r.float()
    ops.set_wide_plan(*plan)
    ops.linear(x, wq, residual=r, w_scale=s)
    close(r, exp_r, 3e-2 * math.sqrt(k / 4096), 1e-2)
    ops.set_wide_plan(*plan)
    a = ops.linear(x, wq, w_scale=s)
    ops.set_wide_plan(*plan)
    b = ops.linear(x, wq, w_scale=s)
    assert torch.equal(a, b)


@pytest.mark.parametrize("plan", [(0, 0), (8, 1), (4, 3)])
@pytest.mark.parametrize("m", [33, 75, 128])
def test_wide_fp8_qkv_rope(plan, m):
    torch.manual_seed(47)
    dt, bs, nb, hq, hkv, H = torch.bfloat16, 16, 64, 8, 1, 8192
    x = torch.randn(m, H, dtype=dt, device="cuda") * 2
    wq, s, deq = _fp8(torch.randn((hq + 2 * hkv) * 128, H, dtype=dt, device="cuda") * 0.02,
                      "qkv")
    pos = torch.randint(0, 4000, (m,), dtype=torch.int32, device="cuda")
    slots = torch.randperm(nb * bs, device="cuda")[:m].to(torch.int32)
    slots[1] = -1
    cs = ref.rope_cos_sin(128, 8192, 500000.0, None, device="cuda")
    k1 = torch.randn(nb, hkv, bs, 128, dtype=dt, device="cuda")
    v1 = torch.randn(nb, hkv, 128, bs, dtype=dt, device="cuda")
    k2, v2 = k1.clone(), v1.clone()
    q_exp = ref.rope_cache(torch.nn.functional.linear(_norm_ref(x).float(), deq).to(dt), pos,
                           slots, cs, k1, v1, hq, hkv, 128)
    ops.set_wide_plan(*plan)
    q_got = ops.decode_qkv_rope(x, wq, 1e-5, pos, slots, cs, k2, v2, hq, hkv, w_scale=s)
    close(q_got, q_exp, 3e-2, 2e-2)
    close(k2, k1, 3e-2, 2e-2)
    close(v2, v1, 3e-2, 2e-2)


@pytest.mark.parametrize("plan", [(0, 0), (8, 2), (4, 1)])
@pytest.mark.parametrize("m", [33, 85, 128])
def test_wide_fp8_gate_up_silu(plan, m):
    torch.manual_seed(48)
    dt, inter, k = torch.bfloat16, 1792, 8192
    x = torch.randn(m, k, dtype=dt, device="cuda")
    wq, s, deq = _fp8(torch.randn(2 * inter, k, dtype=dt, device="cuda") * 0.02, "silu")
    g = _norm_ref(x).float() @ deq.t()
    o32 = torch.nn.functional.silu(g[:, :inter]) * g[:, inter:]
    ops.set_wide_plan(*plan)
    got = ops.decode_gate_up_silu(x, wq, 1e-5, w_scale=s)
    close(got, o32, 6e-2, 4e-2)


def test_wide_fp8_matches_skinny_at_the_seam():
    """fp8: 32 rows (16-row-tile W8 GEMV) and 33 rows (wide W8 build) agree on the first 32."""
    torch.manual_seed(49)
    dt = torch.bfloat16
    x = torch.randn(33, 4096, dtype=dt, device="cuda")
    wq, s, _ = _fp8(torch.randn(4096, 4096, dtype=dt, device="cuda") * 0.02)
    a = ops.linear(x[:32].contiguous(), wq, w_scale=s)
    b = ops.linear(x, wq, w_scale=s)
    close(b[:32], a, 2e-2, 1e-2)


def test_wide_splitk_half_slabs():
    """ATTA_SPLITK_HALF / ops.set_splitk_half: bf16 split-K slabs (half the slab traffic,
    3-10 % per layer at 85-128 rows) round each slice's partial once, so their error vs the fp32
    oracle grows with the partials' magnitude, not the result's (off by default: a cancelling
    row can lose ~1 % relative).  Checked here against the fp32-slab kernel's own error."""
    torch.manual_seed(50)
    dt = torch.bfloat16
    x = torch.randn(85, 4096, dtype=dt, device="cuda")
    w = torch.randn(4096, 4096, dtype=dt, device="cuda") * 0.02
    wp = ops.preshuffle(w)
    exp = x.float() @ w.float().t()
    errs = {}
    try:
        for half in (False, True):
            ops.set_splitk_half(half)
            ops.set_wide_plan(8, 4)
            errs[half] = float((ops.linear(x, wp, preshuffled=True).float() - exp).abs().max())
    finally:
        ops.set_splitk_half(False)
    assert errs[True] <= 4 * errs[False] + 2e-2, errs
