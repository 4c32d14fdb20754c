"""Mid-M GEMM (ops/csrc/midm.h): 129-1000+ rows over pre-shuffled 16-bit weights with the
decode GEMVs' fused epilogues, against the fp32 PyTorch reference (ops/reference.py).  Every
epilogue (plain, residual add, RMSNorm-folded QKV + RoPE + paged K/V write, RMSNorm-folded
gate_up + SiLU-mul), ragged M (129, 200, 382, 475, 512, 640, 1000), every built row-block
height and K split (split-K slices combined in slice order: bitwise deterministic)."""
import math

import pytest
import torch

from agentic_traffic_testing_amd import ops
from agentic_traffic_testing_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
MS = [129, 200, 382, 475, 512, 640, 1000]


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert ops.native_available(), ops._load_error
    ops.ensure_splitk_workspace("cuda")


def close(a, b, atol, rtol=0.0):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    assert bool((err <= tol).all()), f"max err {err.max().item():.4g}"


def _norm_ref(x, eps=1e-5):
    return ref.rms_norm(x, torch.ones(x.shape[1], dtype=x.dtype, device=x.device), eps)


@pytest.mark.parametrize("plan", [(0, 0), (3, 1), (5, 2), (8, 3), (12, 4), (10, 1), (6, 8)])
@pytest.mark.parametrize("m,n,k", [(129, 4096, 4096), (382, 6144, 4096), (475, 4096, 14336),
                                   (200, 1024, 2048), (640, 2048, 4096), (1000, 512, 1024)])
def test_midm_linear_plain_and_residual(plan, m, n, k):
    torch.manual_seed(51)
    dt = torch.bfloat16
    x = torch.randn(m, k, dtype=dt, device="cuda")
    w = torch.randn(n, k, dtype=dt, device="cuda") * 0.02
    wp = ops.preshuffle(w)
    exp = x.float() @ w.float().t()
    assert ops.skinny_ok(x, wp, preshuffled=True)
    ops.set_midm_plan(*plan)
    got = ops.linear(x, wp, preshuffled=True)
    close(got, exp, 2e-2 * math.sqrt(k / 4096), 1e-2)
    r = torch.randn(m, n, dtype=dt, device="cuda")
    exp_r = exp.to(dt).float() + r.float()
    ops.set_midm_plan(*plan)
    out = ops.linear(x, wp, residual=r, preshuffled=True)
    assert out.data_ptr() == r.data_ptr()
    close(r, exp_r, 3e-2 * math.sqrt(k / 4096), 1e-2)
    ops.set_midm_plan(*plan)
    a = ops.linear(x, wp, preshuffled=True)
    ops.set_midm_plan(*plan)
    b = ops.linear(x, wp, preshuffled=True)
    assert torch.equal(a, b)  # slice-ordered combine: run-to-run bit-identical


@pytest.mark.parametrize("plan", [(0, 0), (3, 1), (5, 1), (8, 1)])
@pytest.mark.parametrize("m", MS)
@pytest.mark.parametrize("hq,hkv,H", [(32, 8, 4096), (8, 1, 8192)])
def test_midm_qkv_rope(plan, m, hq, hkv, H):
    torch.manual_seed(52)
    dt, bs, nb = torch.bfloat16, 16, 128
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
    ops.set_midm_plan(*plan)
    q_got = ops.decode_qkv_rope(x, ops.preshuffle(w, "qkv"), 1e-5, pos, slots, cs, k2, v2, hq,
                                hkv, preshuffled=True)
    close(q_got, q_exp, 3e-2, 2e-2)
    close(k2, k1, 3e-2, 2e-2)
    close(v2, v1, 3e-2, 2e-2)


@pytest.mark.parametrize("plan", [(0, 0), (4, 1), (6, 1), (8, 1)])
@pytest.mark.parametrize("m", MS)
@pytest.mark.parametrize("inter,k", [(14336, 4096), (1792, 8192)])
def test_midm_gate_up_silu(plan, m, inter, k):
    torch.manual_seed(53)
    dt = torch.bfloat16
    x = torch.randn(m, k, dtype=dt, device="cuda")
    w = torch.randn(2 * inter, k, dtype=dt, device="cuda") * 0.02
    n = _norm_ref(x)
    exp = ref.silu_and_mul(torch.nn.functional.linear(n, w))
    g = n.float() @ w.float().t()
    o32 = torch.nn.functional.silu(g[:, :inter]) * g[:, inter:]
    ops.set_midm_plan(*plan)
    got = ops.decode_gate_up_silu(x, ops.preshuffle(w, "silu"), 1e-5, preshuffled=True)
    # |silu(g) u| reaches ~10 here, where one bf16 rounding of g or u moves the product by
    # ~0.1: the kernel must be as close to the fp32 oracle as the bf16 library path is
    e_got = float((got.float() - o32).abs().max())
    e_ref = float((exp.float() - o32).abs().max())
    assert e_got <= 1.5 * e_ref + 2e-2, (e_got, e_ref)


def test_midm_fp16_and_seam():
    """fp16 operands, and the 128 / 129-row seam between the wide and mid-M kernels: the first
    128 rows agree to 16-bit rounding."""
    torch.manual_seed(54)
    for dt in (torch.float16, torch.bfloat16):
        x = torch.randn(129, 4096, dtype=dt, device="cuda")
        w = torch.randn(4096, 4096, dtype=dt, device="cuda") * 0.02
        wp = ops.preshuffle(w)
        a = ops.linear(x[:128].contiguous(), wp, preshuffled=True)
        b = ops.linear(x, wp, preshuffled=True)
        close(b[:128], a, 2e-2, 1e-2)
        close(b, x.float() @ w.float().t(), 2e-2, 1e-2)


def test_midm_plan_fills_the_chip():
    """The planned grids of the 8B projections at the burst shapes reach >= 160 workgroups
    (the point of the row-blocked decomposition: the library's 256 x 256 tiles ran 48)."""
    for m in (382, 475):
        for ntiles, k, epi in ((384, 4096, 2), (256, 4096, 1), (1792, 4096, 3), (256, 14336, 1)):
            bmt, s = ops.midm_plan(m, ntiles, k, epi)
            nrb = -(-m // (16 * bmt))
            wgs = nrb * (-(-ntiles // 8)) * s
            assert wgs >= 160, (m, ntiles, k, bmt, s, wgs)
            if epi in (2, 3):
                assert s == 1 and bmt <= 8


# ---- fp8 weights (W8 builds: e4m3fn weight-only, per-row scales) ----------------------------
def _fp8(w, rowmap="plain"):
    q, s = ops.quantize_fp8(w)
    deq = q.view(torch.float8_e4m3fn).float() * s[:, None]
    return ops.preshuffle_fp8(q, rowmap), s, deq


@pytest.mark.parametrize("plan", [(0, 0), (4, 1), (8, 2), (12, 1)])
@pytest.mark.parametrize("m,n,k", [(129, 1024, 8192), (395, 8192, 8192), (640, 2048, 4096)])
def test_midm_fp8_linear_plain_and_residual(plan, m, n, k):
    torch.manual_seed(55)
    dt = torch.bfloat16
    x = torch.randn(m, k, dtype=dt, device="cuda")
    wq, s, deq = _fp8(torch.randn(n, k, dtype=dt, device="cuda") * 0.02)
    exp = x.float() @ deq.t()
    assert ops.skinny_ok(x, wq, preshuffled=True, fp8=True)
    ops.set_midm_plan(*plan)
    got = ops.linear(x, wq, w_scale=s)
    close(got, exp, 2e-2 * math.sqrt(k / 4096), 1e-2)
    r = torch.randn(m, n, dtype=dt, device="cuda")
    exp_r = exp.to(dt).float() + r.float()
    ops.set_midm_plan(*plan)
    ops.linear(x, wq, residual=r, w_scale=s)
    close(r, exp_r, 3e-2 * math.sqrt(k / 4096), 1e-2)


@pytest.mark.parametrize("m", [129, 395, 700])
def test_midm_fp8_qkv_rope_and_gate_up(m):
    torch.manual_seed(56)
    dt, bs, nb, hq, hkv, H, inter = torch.bfloat16, 16, 128, 8, 1, 8192, 1792
    x = torch.randn(m, H, dtype=dt, device="cuda") * 2
    wq, s, deq = _fp8(torch.randn((hq + 2 * hkv) * 128, H, dtype=dt, device="cuda") * 0.02, "qkv")
    pos = torch.randint(0, 4000, (m,), dtype=torch.int32, device="cuda")
    slots = torch.randperm(nb * bs, device="cuda")[:m].to(torch.int32)
    slots[1] = -1
    cs = ref.rope_cos_sin(128, 8192, 500000.0, None, device="cuda")
    k1 = torch.randn(nb, hkv, bs, 128, dtype=dt, device="cuda")
    v1 = torch.randn(nb, hkv, 128, bs, dtype=dt, device="cuda")
    k2, v2 = k1.clone(), v1.clone()
    q_exp = ref.rope_cache(torch.nn.functional.linear(_norm_ref(x).float(), deq).to(dt), pos,
                           slots, cs, k1, v1, hq, hkv, 128)
    q_got = ops.decode_qkv_rope(x, wq, 1e-5, pos, slots, cs, k2, v2, hq, hkv, w_scale=s)
    close(q_got, q_exp, 3e-2, 2e-2)
    close(k2, k1, 3e-2, 2e-2)
    close(v2, v1, 3e-2, 2e-2)
    gq, gs, gdeq = _fp8(torch.randn(2 * inter, H, dtype=dt, device="cuda") * 0.02, "silu")
    g = _norm_ref(x).float() @ gdeq.t()
    o32 = torch.nn.functional.silu(g[:, :inter]) * g[:, inter:]
    close(ops.decode_gate_up_silu(x, gq, 1e-5, w_scale=gs), o32, 6e-2, 4e-2)
