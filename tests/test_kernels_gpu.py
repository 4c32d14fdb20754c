"""HIP kernel numerics vs the fp32 PyTorch reference (ops/reference.py)."""
import math
import os

import numpy as np
import pytest
import torch

from agentic_traffic_testing_amd import ops
from agentic_traffic_testing_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DT = [torch.bfloat16, torch.float16]


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert ops.native_available(), ops._load_error


def close(a, b, atol, rtol=0.0):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    assert bool((err <= tol).all()), f"max err {err.max().item():.4g}"


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("shape", [(1, 4096), (7, 4096), (33, 8192), (300, 1024), (5, 3072),
                                   (2600, 4096), (3, 16384)])
def test_rms_norm(dtype, shape):
    torch.manual_seed(0)
    x = torch.randn(shape, dtype=dtype, device="cuda")
    w = (torch.rand(shape[1], device="cuda") + 0.5).to(dtype)
    close(ops.rms_norm(x, w, 1e-5), ref.rms_norm(x, w, 1e-5), 2e-2, 1e-2)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("shape", [(1, 4096), (9, 4096), (128, 8192), (5, 16384)])
def test_fused_add_rms_norm(dtype, shape):
    torch.manual_seed(1)
    x = torch.randn(shape, dtype=dtype, device="cuda")
    r = torch.randn(shape, dtype=dtype, device="cuda")
    w = (torch.rand(shape[1], device="cuda") + 0.5).to(dtype)
    exp_n, exp_r = ref.fused_add_rms_norm(x, r, w, 1e-5)
    r2 = r.clone()
    got = ops.fused_add_rms_norm(x, r2, w, 1e-5)
    close(r2, exp_r, 0.0)  # residual add is exact up to the same rounding
    close(got, exp_n, 2e-2, 1e-2)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("shape", [(1, 28672), (13, 28672), (64, 7168)])
def test_silu_and_mul(dtype, shape):
    torch.manual_seed(2)
    x = torch.randn(shape, dtype=dtype, device="cuda") * 3
    close(ops.silu_and_mul(x), ref.silu_and_mul(x), 2e-2, 1e-2)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("rows", [1, 5, 16, 300])
def test_embed(dtype, rows):
    torch.manual_seed(3)
    table = torch.randn(1000, 4096, dtype=dtype, device="cuda")
    ids = torch.randint(0, 1000, (rows,), device="cuda", dtype=torch.int32)
    close(ops.embed(table, ids), torch.nn.functional.embedding(ids.long(), table), 0.0)
    # look-ahead mode: the device flag switches the row source to the int64 sample buffer
    prev = torch.randint(0, 1000, (rows + 3,), device="cuda", dtype=torch.int64)
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    close(ops.embed(table, ids, prev, flag), torch.nn.functional.embedding(ids.long(), table), 0.0)
    flag.fill_(1)
    close(ops.embed(table, ids, prev, flag), torch.nn.functional.embedding(prev[:rows], table), 0.0)


def _rand_cache(nb, hkv, bs, d, dtype):
    k = torch.randn(nb, hkv, bs, d, dtype=dtype, device="cuda")
    v = torch.randn(nb, hkv, d, bs, dtype=dtype, device="cuda")
    return k, v


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("hq,hkv", [(32, 8), (8, 1), (4, 1), (24, 8)])
@pytest.mark.parametrize("T", [5, 37, 300])  # < 16: per-token kernel; else 16-token tiles
def test_rope_cache(dtype, hq, hkv, T):
    torch.manual_seed(3)
    D, bs, nb = 128, 16, 64
    qkv = torch.randn(T, (hq + 2 * hkv) * D, dtype=dtype, device="cuda")
    pos = torch.randint(0, 4000, (T,), dtype=torch.int32, device="cuda")
    slots = torch.randperm(nb * bs, device="cuda")[:T].to(torch.int32)
    if T == 300:  # pages filled in order from mid-page (the prefill case the tiles coalesce)
        slots = torch.arange(T, dtype=torch.int32, device="cuda") + 40
    slots[T // 2] = -1
    cs = ref.rope_cos_sin(D, 8192, 500000.0, {"rope_type": "llama3", "factor": 8.0,
                                              "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                              "original_max_position_embeddings": 8192},
                          device="cuda")
    k1, v1 = _rand_cache(nb, hkv, bs, D, dtype)
    k2, v2 = k1.clone(), v1.clone()
    q_exp = ref.rope_cache(qkv, pos, slots, cs, k1, v1, hq, hkv, D)
    q_got = ops.rope_cache(qkv, pos, slots, cs, k2, v2, hq, hkv, D)
    close(q_got, q_exp, 2e-2, 1e-2)
    close(k2, k1, 2e-2, 1e-2)
    close(v2, v1, 0.0)


def _make_paged(seqs, hkv, bs, dtype, nb_extra=8, seed=0):
    """seqs: list of (kvlen, qlen). Returns caches, block tables, metadata on cuda."""
    g = torch.Generator().manual_seed(seed)
    nblk = [math.ceil(kv / bs) for kv, _ in seqs]
    nb = sum(nblk) + nb_extra
    perm = torch.randperm(nb, generator=g)
    W = max(nblk) + 2
    bt = torch.zeros(len(seqs), W, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nblk):
        bt[i, :n] = perm[o:o + n].to(torch.int32)
        bt[i, n:] = -7 if i % 2 else 0  # garbage past the end must never be read
        o += n
    k, v = _rand_cache(nb, hkv, bs, 128, dtype)
    kvlen = torch.tensor([kv for kv, _ in seqs], dtype=torch.int32)
    qlens = [q for _, q in seqs]
    qstart = torch.tensor([0] + list(np.cumsum(qlens)), dtype=torch.int32)
    return k, v, bt.cuda(), kvlen.cuda(), qstart.cuda(), int(sum(qlens))


def _tiles(seqs, tile):
    ts, to = [], []
    for i, (_, ql) in enumerate(seqs):
        for off in range(0, ql, tile):
            ts.append(i)
            to.append(off)
    return (torch.tensor(ts, dtype=torch.int32, device="cuda"),
            torch.tensor(to, dtype=torch.int32, device="cuda"))


@pytest.mark.parametrize("splits", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (24, 8)])
def test_flash_prefill_split_kv(splits, hq, hkv):
    """Split-KV flash prefill (up to `splits` workgroups per (tile, KV head) over contiguous key
    ranges of >= 8 blocks, merged by the last arriver): the cached burst (5 x 17 new tokens over
    617 keys), a planning step over a 176-token prefix, a short fresh prompt, a chunk after a
    prefix, a full causal prompt and short suffixes over 2-4k cached keys (the split cases) -
    against the fp32 reference, run twice (the arrival counters re-arm)."""
    torch.manual_seed(9)
    dt = torch.bfloat16
    seqs = [(617, 17)] * 5 + [(193, 17), (17, 17), (300, 77), (640, 640), (4113, 17),
                                (2100, 40)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, hkv, 16, dt)
    q = torch.randn(T, hq, 128, dtype=dt, device="cuda")
    ts, to = _tiles(seqs, ops.prefill_tile_tokens(hq // hkv, "flash"))
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, k, v, bt.clamp(min=0), kvlen, qstart, scale)
    for _ in range(2):
        got = ops.attention_prefill(q, k, v, bt, kvlen, qstart, ts, to, scale, impl="flash",
                                    kv_splits=splits)
        close(got, exp, 1.5e-2, 2e-2)
    assert int(ops._FLASH_COUNTERS.get(torch.cuda.current_device(),
                                       torch.zeros(1, device="cuda")).abs().sum()) == 0


@pytest.mark.parametrize("impl", ["flash", "v1"])
@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (8, 1), (4, 1), (16, 16), (24, 8)])
@pytest.mark.parametrize("bs", [16, 32])
def test_attention_prefill(impl, dtype, hq, hkv, bs):
    torch.manual_seed(4)
    # (kvlen, qlen): full prompt, chunk after cached prefix, single token, long-ish
    seqs = [(53, 53), (300, 77), (17, 1), (640, 640), (129, 2)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, hkv, bs, dtype)
    q = torch.randn(T, hq, 128, dtype=dtype, device="cuda")
    ts, to = _tiles(seqs, ops.prefill_tile_tokens(hq // hkv, impl))
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, k, v, bt.clamp(min=0), kvlen, qstart, scale)
    got = ops.attention_prefill(q, k, v, bt, kvlen, qstart, ts, to, scale, impl=impl)
    close(got, exp, 1.5e-2, 2e-2)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (8, 1), (24, 8), (16, 16)])
def test_flash_prefill_8_waves_bit_identical(dtype, hq, hkv):
    """8-wave flash-prefill workgroups (waves 0-3 stage K, 4-7 stage V; 256 columns per staged
    block) compute every column with the same keys in the same order as the 4-wave kernel:
    bit-identical outputs, and within tolerance of the fp32 reference."""
    torch.manual_seed(8)
    seqs = [(53, 53), (300, 77), (17, 1), (900, 900), (129, 2), (2000, 150)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, hkv, 16, dtype)
    q = torch.randn(T, hq, 128, dtype=dtype, device="cuda")
    scale = 1 / math.sqrt(128)
    outs = {}
    try:
        for nw in (4, 8):
            ops.set_flash_waves(nw)
            ts, to = _tiles(seqs, ops.prefill_tile_tokens(hq // hkv, "flash"))
            # unsplit: the 4- and 8-wave tiles differ in size, so an automatic split-KV plan
            # (per tile count) would sum different key ranges (test_flash_prefill_split_kv)
            outs[nw] = ops.attention_prefill(q, k, v, bt, kvlen, qstart, ts, to, scale,
                                             impl="flash", kv_splits=1)
    finally:
        ops.set_flash_waves(int(os.environ.get("ATTA_FLASH_WAVES", "4")))
    assert torch.equal(outs[4], outs[8])
    exp = ref.paged_attention(q, k, v, bt.clamp(min=0), kvlen, qstart, scale)
    close(outs[8], exp, 1.5e-2, 2e-2)


@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (24, 8)])
def test_flash_prefill_long_chunked(hq, hkv):
    """2.6k-token prompt (the fan-out synthesis size) plus a chunk after a 3k cached prefix
    and an 11k-context chunk (reference .env max_model_len 11000): the flash kernel's block
    loop, diagonal masking and block-table staging stay exact."""
    torch.manual_seed(6)
    dt = torch.bfloat16
    seqs = [(2600, 2600), (3000 + 700, 700), (11000, 300)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, hkv, 16, dt)
    q = torch.randn(T, hq, 128, dtype=dt, device="cuda")
    ts, to = _tiles(seqs, ops.prefill_tile_tokens(hq // hkv, "flash"))
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, k, v, bt.clamp(min=0), kvlen, qstart, scale)
    got = ops.attention_prefill(q, k, v, bt, kvlen, qstart, ts, to, scale, impl="flash")
    close(got, exp, 1.5e-2, 2e-2)


@pytest.mark.parametrize("qscale", [6.0, 24.0])
@pytest.mark.parametrize("bs", [16, 32])
def test_flash_prefill_large_logits(qscale, bs):
    """Scores spread over tens of log2 units, so running maxima keep growing past the
    defer-max threshold: the kernel's rescale of O and l (taken only when a column's max grew
    by more than 2^8) and its stale-max blocks must still match the fp32 reference."""
    torch.manual_seed(7)
    dt = torch.bfloat16
    seqs = [(700, 700), (1500, 400)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, 8, bs, dt)
    q = (torch.randn(T, 32, 128, device="cuda") * qscale).to(dt)
    ts, to = _tiles(seqs, ops.prefill_tile_tokens(4, "flash"))
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, k, v, bt.clamp(min=0), kvlen, qstart, scale)
    got = ops.attention_prefill(q, k, v, bt, kvlen, qstart, ts, to, scale, impl="flash")
    close(got, exp, 1.5e-2, 2e-2)


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("hq,hkv", [(32, 8), (64, 8), (8, 1), (4, 1), (24, 8)])
@pytest.mark.parametrize("parts", [1, 4, 16])
def test_attention_decode(dtype, hq, hkv, parts):
    torch.manual_seed(5)
    bs = 16
    seqs = [(1, 1), (17, 1), (256, 1), (1000, 1), (63, 1), (2048, 1)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, hkv, bs, dtype)
    q = torch.randn(T, hq, 128, dtype=dtype, device="cuda")
    part_tokens = 64 * math.ceil(2048 / parts / 64) if parts > 1 else 2048
    nparts = math.ceil(2048 / part_tokens)
    po = torch.empty(len(seqs) * hkv * nparts * 16 * 128, device="cuda")
    pl = torch.empty(len(seqs) * hkv * nparts * 16, device="cuda")
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, k, v, bt.clamp(min=0), kvlen, qstart, scale)
    got = ops.attention_decode(q, k, v, bt, kvlen, qstart, scale, po, pl, nparts, part_tokens)
    close(got, exp, 1.5e-2, 2e-2)


def test_attention_decode_padded_and_subset():
    """Dummy (kvlen 0) sequences and num_seqs < S must not touch other rows."""
    dtype = torch.bfloat16
    seqs = [(40, 1), (90, 1), (1, 1)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, 8, 16, dtype)
    kvlen[2] = 0
    q = torch.randn(T, 32, 128, dtype=dtype, device="cuda")
    out = torch.full_like(q, 7.0)
    po = torch.empty(3 * 8 * 4 * 16 * 128, device="cuda")
    pl = torch.empty(3 * 8 * 4 * 16, device="cuda")
    ops.attention_decode(q, k, v, bt, kvlen, qstart, 0.088, po, pl, 4, 64, out=out, num_seqs=1)
    exp = ref.paged_attention(q, k, v, bt, kvlen, qstart, 0.088)
    close(out[0], exp[0], 1.5e-2, 2e-2)
    assert bool((out[1:] == 7.0).all())
    ops.attention_decode(q, k, v, bt, kvlen, qstart, 0.088, po, pl, 4, 64, out=out)
    assert bool((out[2] == 0).all())


def test_attention_softmax_spike():
    """A huge score on one key forces the running max to jump mid-sequence."""
    dtype = torch.bfloat16
    seqs = [(700, 700)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, 8, 16, dtype)
    q = torch.randn(T, 32, 128, dtype=dtype, device="cuda") * 0.1
    page = int(bt[0, 500 // 16])
    k[page, :, 500 % 16, :] = 6.0
    q[600:, :, :] = 1.0
    tiles = torch.arange(0, 700, 16, dtype=torch.int32, device="cuda")
    ts = torch.zeros_like(tiles)
    exp = ref.paged_attention(q, k, v, bt, kvlen, qstart, 1 / math.sqrt(128))
    got = ops.attention_prefill(q, k, v, bt, kvlen, qstart, ts, tiles, 1 / math.sqrt(128))
    close(got, exp, 1.5e-2, 2e-2)


def test_sample_greedy_and_gumbel():
    torch.manual_seed(6)
    B, V = 6, 128256
    logits = torch.randn(B, V, device="cuda") * 3
    temp = torch.tensor([0.0, 0.2, 1.0, 0.0, 0.7, 2.0], device="cuda")
    seeds = torch.arange(B, dtype=torch.int64, device="cuda") * 977 + 11
    steps = torch.arange(B, dtype=torch.int64, device="cuda") * 3
    got = ops.sample(logits, temp, seeds, steps).cpu()
    exp = ref.sample(logits.cpu(), temp.cpu(), seeds.cpu(), steps.cpu())
    assert got[0] == exp[0] and got[3] == exp[3]
    # fast-math logs may flip near-ties; the bulk must agree
    assert int((got == exp).sum()) >= B - 1
    # bf16 logits path
    got16 = ops.sample(logits.to(torch.bfloat16), temp, seeds, steps).cpu()
    assert got16[0] == int(torch.argmax(logits[0].to(torch.bfloat16).float()))


def test_sample_distribution():
    """Gumbel-max draws follow softmax(logits / T)."""
    V, N = 16, 4000
    logits = torch.linspace(-2, 2, V, device="cuda").repeat(N, 1)
    temp = torch.full((N,), 0.8, device="cuda")
    seeds = torch.full((N,), 42, dtype=torch.int64, device="cuda")
    steps = torch.arange(N, dtype=torch.int64, device="cuda")
    toks = ops.sample(logits, temp, seeds, steps).cpu()
    freq = torch.bincount(toks, minlength=V).float() / N
    p = torch.softmax(logits[0].cpu() / 0.8, -1)
    assert float((freq - p).abs().max()) < 0.03


def test_sample_topkp_matches_reference():
    """Native top-k / top-p sampler vs the reference definition (exact radix-select
    thresholds, same Gumbel draw); rows with both filters off == the plain sampler."""
    torch.manual_seed(8)
    B, V = 12, 128256
    logits = torch.randn(B, V, device="cuda") * 3
    logits[5, 100:110] = 9.0  # a tie group straddling the top-k / top-p boundary
    temp = torch.tensor([0.5, 0.2, 1.0, 0.0, 0.7, 1.0, 0.5, 2.0, 0.5, 1.0, 0.25, 1.0],
                        device="cuda")
    top_p = torch.tensor([1.0, 0.9, 0.5, 0.9, 1.0, 0.95, 0.1, 0.99, 1.0, 0.0, 0.8, 1.0],
                         device="cuda")
    top_k = torch.tensor([0, 0, 0, 5, 50, 4, -1, 1000, 1, 20, 128255, 128256],
                         dtype=torch.int32, device="cuda")
    seeds = torch.arange(B, dtype=torch.int64, device="cuda") * 131 + 7
    steps = torch.arange(B, dtype=torch.int64, device="cuda") * 5
    got = ops.sample_topkp(logits, temp, top_p, top_k, seeds, steps).cpu()
    exp = ref.sample_topkp(logits.cpu(), temp.cpu(), top_p.cpu(), top_k.cpu(), seeds.cpu(),
                           steps.cpu())
    # fast-math Gumbel logs may flip a near-tie; the bulk must agree
    assert int((got == exp).sum()) >= B - 1, (got, exp)
    # top-k = 1 and top-p = 0 are argmax whatever the noise
    assert int(got[8]) == int(torch.argmax(logits[8])) and int(got[9]) == int(torch.argmax(logits[9]))
    # both filters off: bit-identical to the plain sampler (same noise, same tie-break)
    plain = ops.sample(logits, temp, seeds, steps).cpu()
    for r in (0, 11):
        assert int(got[r]) == int(plain[r])
    # bf16 logits, deterministic
    l16 = logits.to(torch.bfloat16)
    a = ops.sample_topkp(l16, temp, top_p, top_k, seeds, steps).cpu()
    b = ops.sample_topkp(l16, temp, top_p, top_k, seeds, steps).cpu()
    assert torch.equal(a, b)


def test_sample_topkp_distribution():
    """Draws stay inside the kept set and follow the renormalised softmax over it."""
    V, N = 16, 6000
    logits = torch.linspace(-2, 2, V, device="cuda").repeat(N, 1)
    temp = torch.full((N,), 0.8, device="cuda")
    seeds = torch.full((N,), 42, dtype=torch.int64, device="cuda")
    steps = torch.arange(N, dtype=torch.int64, device="cuda")
    p = torch.softmax(logits[0].cpu() / 0.8, -1)
    # top-k 4: the 4 largest
    toks = ops.sample_topkp(logits, temp, torch.ones(N, device="cuda"),
                            torch.full((N,), 4, dtype=torch.int32, device="cuda"), seeds,
                            steps).cpu()
    freq = torch.bincount(toks, minlength=V).float() / N
    assert float(freq[:12].sum()) == 0.0
    q = p.clone()
    q[:12] = 0
    q /= q.sum()
    assert float((freq - q).abs().max()) < 0.03
    # top-p 0.7: smallest top set with mass >= 0.7
    toks = ops.sample_topkp(logits, temp, torch.full((N,), 0.7, device="cuda"),
                            torch.zeros(N, dtype=torch.int32, device="cuda"), seeds, steps).cpu()
    order = torch.argsort(p, descending=True)
    n_keep = int((torch.cumsum(p[order], 0) < 0.7).sum()) + 1
    keep = order[:n_keep]
    freq = torch.bincount(toks, minlength=V).float() / N
    mask = torch.zeros(V, dtype=torch.bool)
    mask[keep] = True
    assert float(freq[~mask].sum()) == 0.0
    q = torch.where(mask, p, torch.zeros(()))
    q /= q.sum()
    assert float((freq - q).abs().max()) < 0.03


@pytest.mark.parametrize("dtype", DT)
@pytest.mark.parametrize("m,n,k", [(1, 6144, 4096), (5, 4096, 4096), (12, 28672, 4096),
                                   (16, 4096, 14336), (3, 128256, 4096), (24, 1024, 3584),
                                   (64, 512, 8192)])
def test_skinny_gemm(dtype, m, n, k):
    torch.manual_seed(7)
    x = torch.randn(m, k, dtype=dtype, device="cuda")
    w = torch.randn(n, k, dtype=dtype, device="cuda") * 0.02
    exp = (x.float() @ w.float().t())
    got = ops.linear(x, w)
    close(got, exp, 2e-2 * math.sqrt(k / 4096), 1e-2)
    r = torch.randn(m, n, dtype=dtype, device="cuda")
    exp_r = (exp.to(dtype).float() + r.float())
    got_r = ops.linear(x, w, residual=r)  # in place on r
    assert got_r.data_ptr() == r.data_ptr()
    close(got_r, exp_r, 3e-2 * math.sqrt(k / 4096), 1e-2)


@pytest.mark.parametrize("ksplit", [2, 4])
@pytest.mark.parametrize("m,n,k", [(1, 1280, 8192), (5, 4096, 4096), (20, 2048, 14336)])
def test_skinny_gemm_splitk(ksplit, m, n, k):
    """Split-K GEMV (in-launch combine of fp32 slice partials by the last arriving slice)
    vs the fp32 reference, plain and residual epilogues, repeated so counters must re-arm."""
    torch.manual_seed(17)
    dt = torch.bfloat16
    x = torch.randn(m, k, dtype=dt, device="cuda")
    w = torch.randn(n, k, dtype=dt, device="cuda") * 0.02
    wp = ops.preshuffle(w)
    exp = x.float() @ w.float().t()
    for _ in range(3):
        got = ops.linear(x, wp, waves=4, preshuffled=True, ksplit=ksplit)
        close(got, exp, 2e-2 * math.sqrt(k / 4096), 1e-2)
        r = torch.randn(m, n, dtype=dt, device="cuda")
        exp_r = exp.to(dt).float() + r.float()
        ops.linear(x, wp, residual=r, waves=8, preshuffled=True, ksplit=ksplit)
        close(r, exp_r, 3e-2 * math.sqrt(k / 4096), 1e-2)
    ws, counters = ops._SPLITK_WS[torch.cuda.current_device()]
    assert bool((counters == 0).all())
    # slice partials are summed in slice order: the result is run-to-run bit-identical
    a = ops.linear(x, wp, waves=4, preshuffled=True, ksplit=ksplit)
    b = ops.linear(x, wp, waves=4, preshuffled=True, ksplit=ksplit)
    assert torch.equal(a, b)


@pytest.mark.parametrize("ksplit", [2, 4])
def test_fused_decode_kernels_splitk(ksplit):
    """Fused qkv+RoPE and gate_up+SiLU epilogues (RMSNorm row sums combined across slices)."""
    torch.manual_seed(19)
    dt, H, bs, nb, hq, hkv, m = torch.bfloat16, 8192, 16, 64, 8, 1, 5
    x = torch.randn(m, H, dtype=dt, device="cuda") * 2
    w = torch.randn((hq + 2 * hkv) * 128, H, dtype=dt, device="cuda") * 0.02
    pos = torch.randint(0, 4000, (m,), dtype=torch.int32, device="cuda")
    slots = torch.randperm(nb * bs, device="cuda")[:m].to(torch.int32)
    cs = ref.rope_cos_sin(128, 8192, 500000.0, None, device="cuda")
    k1, v1 = _rand_cache(nb, hkv, bs, 128, dt)
    k2, v2 = k1.clone(), v1.clone()
    q_exp = ref.rope_cache(torch.nn.functional.linear(_norm_ref(x), w), pos, slots, cs, k1, v1,
                           hq, hkv, 128)
    q_got = ops.decode_qkv_rope(x, ops.preshuffle(w, "qkv"), 1e-5, pos, slots, cs, k2, v2, hq,
                                hkv, preshuffled=True, ksplit=ksplit)
    close(q_got, q_exp, 3e-2, 2e-2)
    close(k2, k1, 3e-2, 2e-2)
    close(v2, v1, 3e-2, 2e-2)
    inter = 1024
    wg = torch.randn(2 * inter, H, dtype=dt, device="cuda") * 0.02
    exp = ref.silu_and_mul(torch.nn.functional.linear(_norm_ref(x), wg))
    got = ops.decode_gate_up_silu(x, ops.preshuffle(wg, "silu"), 1e-5, preshuffled=True,
                                  ksplit=ksplit)
    close(got, exp, 4e-2, 4e-2)


def _norm_ref(x, eps=1e-5):
    return ref.rms_norm(x, torch.ones(x.shape[1], dtype=x.dtype, device=x.device), eps)


@pytest.mark.parametrize("m", [1, 5, 16, 24])
@pytest.mark.parametrize("hq,hkv", [(32, 8), (8, 1), (24, 8)])
def test_decode_qkv_rope(m, hq, hkv):
    torch.manual_seed(8)
    dt, H, bs, nb = torch.bfloat16, 4096, 16, 64
    x = torch.randn(m, H, dtype=dt, device="cuda") * 2
    w = torch.randn((hq + 2 * hkv) * 128, H, dtype=dt, device="cuda") * 0.02
    pos = torch.randint(0, 4000, (m,), dtype=torch.int32, device="cuda")
    slots = torch.randperm(nb * bs, device="cuda")[:m].to(torch.int32)
    if m > 1:
        slots[1] = -1
    cs = ref.rope_cos_sin(128, 8192, 500000.0, None, device="cuda")
    k1, v1 = _rand_cache(nb, hkv, bs, 128, dt)
    k2, v2 = k1.clone(), v1.clone()
    qkv = torch.nn.functional.linear(_norm_ref(x), w)
    q_exp = ref.rope_cache(qkv, pos, slots, cs, k1, v1, hq, hkv, 128)
    q_got = ops.decode_qkv_rope(x, w, 1e-5, pos, slots, cs, k2, v2, hq, hkv)
    close(q_got, q_exp, 3e-2, 2e-2)
    close(k2, k1, 3e-2, 2e-2)
    close(v2, v1, 3e-2, 2e-2)


@pytest.mark.parametrize("m", [1, 5, 16, 32])
@pytest.mark.parametrize("inter,k", [(14336, 4096), (2816, 1024)])
def test_decode_gate_up_silu(m, inter, k):
    torch.manual_seed(9)
    dt = torch.bfloat16
    x = torch.randn(m, k, dtype=dt, device="cuda")
    w = torch.randn(2 * inter, k, dtype=dt, device="cuda") * 0.02
    exp = ref.silu_and_mul(torch.nn.functional.linear(_norm_ref(x), w))
    got = ops.decode_gate_up_silu(x, w, 1e-5)
    # the kernel scales by 1/rms after the GEMM instead of rounding the normalised row to
    # bf16 first; silu(g)*u then amplifies that last-bit difference
    close(got, exp, 4e-2, 4e-2)


@pytest.mark.parametrize("m", [1, 5, 12])
def test_decode_lm_head_sample(m):
    torch.manual_seed(10)
    dt, V, H = torch.bfloat16, 32768, 1024
    x = torch.randn(m, H, dtype=dt, device="cuda")
    w = torch.randn(V, H, dtype=dt, device="cuda") * 0.05
    keys = torch.full((32 * V // 16,), -1, dtype=torch.int64, device="cuda")  # garbage scratch
    temp = torch.zeros(m, device="cuda")
    seeds = torch.arange(m, dtype=torch.int64, device="cuda")
    steps = torch.zeros(m, dtype=torch.int64, device="cuda")
    logits = torch.nn.functional.linear(_norm_ref(x), w).float()
    for _ in range(3):  # repeated launches reuse the scratch
        got = ops.decode_lm_head_sample(x, w, 1e-5, temp, seeds, steps, keys)
        top2 = torch.topk(logits, 2, dim=-1)
        for r in range(m):
            g = int(got[r])
            # exact argmax unless the top-2 are within bf16 rounding of each other
            assert g == int(top2.indices[r, 0]) or \
                float(top2.values[r, 0] - logits[r, g]) < 0.05
    temp.fill_(0.8)
    toks = ops.decode_lm_head_sample(x, w, 1e-5, temp, seeds, steps, keys)
    assert bool(((toks >= 0) & (toks < V)).all())


@pytest.mark.parametrize("m", [1, 7])
def test_decode_lm_head_sample_vocab_parallel(m):
    """TP path: two vocab shards emit signed-orderable keys (global ids for the noise);
    their MAX must equal sampling over the full vocabulary."""
    torch.manual_seed(12)
    dt, V, H = torch.bfloat16, 8192, 1024
    x = torch.randn(m, H, dtype=dt, device="cuda")
    w = torch.randn(V, H, dtype=dt, device="cuda") * 0.05
    keys = torch.empty(m * V // 16, dtype=torch.int64, device="cuda")
    temp = torch.full((m,), 0.7, device="cuda")
    temp[0] = 0.0
    seeds = torch.arange(m, dtype=torch.int64, device="cuda") + 5
    steps = torch.full((m,), 3, dtype=torch.int64, device="cuda")
    full = ops.decode_lm_head_sample(x, w, 1e-5, temp, seeds, steps, keys).clone()
    shard = V // 2
    k0 = ops.decode_lm_head_sample(x, w[:shard].contiguous(), 1e-5, temp, seeds, steps, keys,
                                   finalize="key", vocab_offset=0).clone()
    k1 = ops.decode_lm_head_sample(x, w[shard:].contiguous(), 1e-5, temp, seeds, steps, keys,
                                   finalize="key", vocab_offset=shard).clone()
    got = ops.key_to_token(torch.maximum(k0, k1))
    assert got.tolist() == full.tolist()
    # keys agree with the fp32 reference's packing on the greedy row
    logits = torch.nn.functional.linear(_norm_ref(x), w).float().cpu()
    ref_keys = ref.sample_keys(logits[:1, shard:], temp[:1].cpu(), seeds[:1].cpu(),
                               steps[:1].cpu(), vocab_offset=shard)
    assert int(ops.key_to_token(ref_keys)[0]) == int(ops.key_to_token(k1[:1])[0]) or \
        abs(float(logits[0, int(ops.key_to_token(k1[:1])[0])]) -
            float(logits[0, int(ops.key_to_token(ref_keys)[0])])) < 0.05


@pytest.mark.parametrize("hq,hkv", [(32, 8), (8, 1), (64, 8), (24, 8)])
@pytest.mark.parametrize("part_tokens", [128, 256, 512])
def test_attention_decode_v2(hq, hkv, part_tokens):
    torch.manual_seed(11)
    dt, bs = torch.bfloat16, 16
    seqs = [(1, 1), (17, 1), (256, 1), (1000, 1), (63, 1), (2048, 1), (0, 1)]
    k, v, bt, kvlen, qstart, T = _make_paged([(max(kv, 1), q) for kv, q in seqs], hkv, bs, dt)
    kvlen[-1] = 0  # dummy (graph padding) sequence
    q = torch.randn(T, hq, 128, dtype=dt, device="cuda")
    max_parts = math.ceil(4096 / part_tokens)
    S = len(seqs)
    po = torch.empty(S * hkv * max_parts * 16 * 128, device="cuda")
    pl = torch.empty(S * hkv * max_parts * 16, device="cuda")
    cnt = torch.zeros(S * hkv, dtype=torch.int32, device="cuda")
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, k, v, bt.clamp(min=0), kvlen, qstart, scale)
    for _ in range(3):  # counters must re-arm
        out = torch.full_like(q, 3.0)
        ops.attention_decode_v2(q, k, v, bt, kvlen, qstart, scale, po, pl, cnt, max_parts,
                                part_tokens, out=out)
        close(out[:-1], exp[:-1], 1.5e-2, 2e-2)
        assert bool((cnt == 0).all())


def _poison_tails(k, v, bt, kvlen, bs, used_pages):
    """Every cache slot no sequence owns - the tail slots of each sequence's last page and
    the unused pages - gets Inf / NaN (the kernels must not rely on a finite,
    zero-initialised cache past a sequence's end)."""
    kv = kvlen.cpu().tolist()
    btc = bt.cpu()
    for i, n in enumerate(kv):
        if n % bs:
            pg = int(btc[i, (n - 1) // bs])
            k[pg, :, n % bs:, :] = float("inf")
            v[pg, :, :, n % bs:] = float("nan")
    free = [p for p in range(k.shape[0]) if p not in used_pages]
    for p in free:
        k[p] = float("nan")
        v[p] = float("inf")


def test_attention_kernels_ignore_nonfinite_stale_slots():
    """Inf / NaN in cache slots past every sequence's end: flash and v1 prefill, the
    two-kernel decode and the in-kernel-combine decode all stay finite and exact."""
    torch.manual_seed(21)
    dt, bs, hq, hkv = torch.bfloat16, 16, 32, 8
    seqs = [(53, 53), (300, 77), (17, 1), (130, 2)]
    k, v, bt, kvlen, qstart, T = _make_paged(seqs, hkv, bs, dt)
    used = {int(bt[i, j]) for i, (kv, _) in enumerate(seqs) for j in range(math.ceil(kv / bs))}
    q = torch.randn(T, hq, 128, dtype=dt, device="cuda")
    scale = 1 / math.sqrt(128)
    exp = ref.paged_attention(q, k, v, bt.clamp(min=0), kvlen, qstart, scale)
    _poison_tails(k, v, bt, kvlen, bs, used)
    bt0 = bt.clamp(min=0)  # page 0 is a real page here: its tail may be poisoned too
    for impl in ("flash", "v1"):
        ts, to = _tiles(seqs, ops.prefill_tile_tokens(hq // hkv, impl))
        got = ops.attention_prefill(q, k, v, bt0, kvlen, qstart, ts, to, scale, impl=impl)
        assert bool(torch.isfinite(got).all()), impl
        close(got, exp, 1.5e-2, 2e-2)
    # decode: one query row per sequence (the last prompt token)
    dseqs = [(kv, 1) for kv, _ in seqs]
    qd = torch.stack([q[int(qstart[i + 1]) - 1] for i in range(len(seqs))])
    qs_d = torch.arange(len(seqs) + 1, dtype=torch.int32, device="cuda")
    exp_d = torch.stack([exp[int(qstart[i + 1]) - 1] for i in range(len(seqs))])
    S = len(dseqs)
    po = torch.empty(S * hkv * 8 * 16 * 128, device="cuda")
    pl = torch.empty(S * hkv * 8 * 16, device="cuda")
    got = ops.attention_decode(qd, k, v, bt0, kvlen, qs_d, scale, po, pl, 4, 128)
    assert bool(torch.isfinite(got).all())
    close(got, exp_d, 1.5e-2, 2e-2)
    cnt = torch.zeros(S * hkv, dtype=torch.int32, device="cuda")
    out = torch.empty_like(qd)
    ops.attention_decode_v2(qd, k, v, bt0, kvlen, qs_d, scale, po, pl, cnt, 8, 128, out=out)
    assert bool(torch.isfinite(out).all())
    close(out, exp_d, 1.5e-2, 2e-2)


def test_attention_decode_v2_grid_invariant():
    """The partition grid (decode graphs are captured per partition bucket) must not change a
    single bit: a grid of exactly the partitions needed, one more, and max_model_len's."""
    torch.manual_seed(12)
    dt, bs, hq, hkv = torch.bfloat16, 16, 32, 8
    seqs = [(510, 1), (1025, 1), (264, 1), (54, 1)]
    k, v, bt, kvlen, qstart, T = _make_paged([(kv, q) for kv, q in seqs], hkv, bs, dt)
    q = torch.randn(T, hq, 128, dtype=dt, device="cuda")
    S, scale = len(seqs), 1 / math.sqrt(128)
    outs = []
    for max_parts in (5, 6, 8, 32):
        po = torch.full((S * hkv * max_parts * 16 * 128,), float("nan"), device="cuda")
        pl = torch.full((S * hkv * max_parts * 16,), float("nan"), device="cuda")
        cnt = torch.zeros(S * hkv, dtype=torch.int32, device="cuda")
        out = torch.full_like(q, 3.0)
        ops.attention_decode_v2(q, k, v, bt, kvlen, qstart, scale, po, pl, cnt, max_parts, 256,
                                out=out)
        torch.cuda.synchronize()
        outs.append(out)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])


@pytest.mark.parametrize("m", [1, 5, 20])
def test_preshuffled_decode_kernels_bit_identical(m, monkeypatch):
    """Pre-shuffled weights feed the same lanes the same products in the same order, so every
    fused decode kernel must return bit-identical results to the row-major layout (at the same
    wave count: the tuned table may split K differently per layout)."""
    monkeypatch.setattr(ops, "DECODE_WAVES",
                        {k: {"rm": v["rm"], "ps": v["rm"], "fp8": v["fp8"]}
                         for k, v in ops.DECODE_WAVES.items()})
    monkeypatch.setattr(ops, "DECODE_WAVES_MT2", {})
    ops.set_wide_min_rows(33, 33)  # 17-32 pre-shuffled rows would run the wide kernel
    try:
        _preshuffled_bit_identical(m)
    finally:
        ops.set_wide_min_rows()


def _preshuffled_bit_identical(m):
    torch.manual_seed(21)
    dt, H, bs = torch.bfloat16, 1024, 16
    x = torch.randn(m, H, dtype=dt, device="cuda")
    # plain GEMM + residual
    w = torch.randn(2048, H, dtype=dt, device="cuda") * 0.05
    wp = ops.preshuffle(w)
    assert torch.equal(ops.linear(x, w), ops.linear(x, wp, preshuffled=True))
    r1 = torch.randn(m, 2048, dtype=dt, device="cuda")
    r2 = r1.clone()
    ops.linear(x, w, residual=r1)
    ops.linear(x, wp, residual=r2, preshuffled=True)
    assert torch.equal(r1, r2)
    # gate_up + SiLU
    inter = 512
    wg = torch.randn(2 * inter, H, dtype=dt, device="cuda") * 0.05
    a = ops.decode_gate_up_silu(x, wg, 1e-5)
    b = ops.decode_gate_up_silu(x, ops.preshuffle(wg, "silu"), 1e-5, preshuffled=True)
    assert torch.equal(a, b)
    # qkv + RoPE + paged KV write
    hq, hkv = 8, 2
    wq = torch.randn((hq + 2 * hkv) * 128, H, dtype=dt, device="cuda") * 0.05
    nb = 8
    kc1 = torch.zeros(nb, hkv, bs, 128, dtype=dt, device="cuda")
    vc1 = torch.zeros(nb, hkv, 128, bs, dtype=dt, device="cuda")
    kc2, vc2 = kc1.clone(), vc1.clone()
    pos = torch.arange(m, dtype=torch.int32, device="cuda") + 3
    slots = torch.arange(m, dtype=torch.int32, device="cuda") * 5
    cs = ref.rope_cos_sin(128, 64, 500000.0, None, device="cuda")
    q1 = ops.decode_qkv_rope(x, wq, 1e-5, pos, slots, cs, kc1, vc1, hq, hkv)
    q2 = ops.decode_qkv_rope(x, ops.preshuffle(wq, "qkv"), 1e-5, pos, slots, cs, kc2, vc2, hq,
                             hkv, preshuffled=True)
    assert torch.equal(q1, q2) and torch.equal(kc1, kc2) and torch.equal(vc1, vc2)
    # LM head + sampler
    V = 4096
    wl = torch.randn(V, H, dtype=dt, device="cuda") * 0.05
    keys = torch.empty(m * V // 16, dtype=torch.int64, device="cuda")
    temp = torch.full((m,), 0.5, device="cuda")
    seeds = torch.arange(m, dtype=torch.int64, device="cuda")
    steps = torch.zeros(m, dtype=torch.int64, device="cuda")
    t1 = ops.decode_lm_head_sample(x, wl, 1e-5, temp, seeds, steps, keys).clone()
    t2 = ops.decode_lm_head_sample(x, ops.preshuffle(wl), 1e-5, temp, seeds, steps, keys,
                                   preshuffled=True)
    assert torch.equal(t1, t2)


@pytest.mark.parametrize("m", [1, 5, 20])
def test_fp8_decode_kernels(m):
    """fp8 weight-only GEMVs (uint8 e4m3fn, per-row scale, pre-shuffled) against the same
    kernels on the dequantised 16-bit weights."""
    torch.manual_seed(31)
    dt, H = torch.bfloat16, 1024
    x = torch.randn(m, H, dtype=dt, device="cuda")

    def q(w, rowmap="plain"):
        qw, sc = ops.quantize_fp8(w)
        return ops.preshuffle_fp8(qw, rowmap), sc, ops.dequantize_fp8(qw, sc, dt)

    w = torch.randn(2048, H, dtype=dt, device="cuda") * 0.05
    wq, sc, wd = q(w)
    close(ops.linear(x, wq, w_scale=sc), ops.linear(x, wd), 2e-2, 2e-2)
    r1 = torch.randn(m, 2048, dtype=dt, device="cuda")
    r2 = r1.clone()
    ops.linear(x, wq, residual=r1, w_scale=sc)
    ops.linear(x, wd, residual=r2)
    close(r1, r2, 3e-2, 2e-2)
    inter = 512
    wg = torch.randn(2 * inter, H, dtype=dt, device="cuda") * 0.05
    gq, gs, gd = q(wg, "silu")
    close(ops.decode_gate_up_silu(x, gq, 1e-5, w_scale=gs), ops.decode_gate_up_silu(x, gd, 1e-5),
          3e-2, 3e-2)
    hq, hkv, bs, nb = 8, 2, 16, 8
    wqkv = torch.randn((hq + 2 * hkv) * 128, H, dtype=dt, device="cuda") * 0.05
    kq, ks, kd = q(wqkv, "qkv")
    kc1 = torch.zeros(nb, hkv, bs, 128, dtype=dt, device="cuda")
    vc1 = torch.zeros(nb, hkv, 128, bs, dtype=dt, device="cuda")
    kc2, vc2 = kc1.clone(), vc1.clone()
    pos = torch.arange(m, dtype=torch.int32, device="cuda")
    slots = torch.arange(m, dtype=torch.int32, device="cuda")
    cs = ref.rope_cos_sin(128, 64, 500000.0, None, device="cuda")
    q1 = ops.decode_qkv_rope(x, kq, 1e-5, pos, slots, cs, kc1, vc1, hq, hkv, w_scale=ks)
    q2 = ops.decode_qkv_rope(x, kd, 1e-5, pos, slots, cs, kc2, vc2, hq, hkv)
    close(q1, q2, 3e-2, 3e-2)
    close(kc1, kc2, 3e-2, 3e-2)
    close(vc1, vc2, 3e-2, 3e-2)
    # down-proj shape with K not a multiple of 1024 (fp8 wave fitting)
    wd2 = torch.randn(256, 3584, dtype=dt, device="cuda") * 0.05
    a = torch.randn(m, 3584, dtype=dt, device="cuda")
    dq, dsc, dd = q(wd2)
    close(ops.linear(a, dq, w_scale=dsc), ops.linear(a, dd), 3e-2, 2e-2)


def test_fp8_prefill_linear():
    torch.manual_seed(32)
    x = torch.randn(300, 1024, dtype=torch.bfloat16, device="cuda")
    w = torch.randn(512, 1024, dtype=torch.bfloat16, device="cuda") * 0.05
    qw, sc = ops.quantize_fp8(w)
    got = ops.linear_fp8(x, qw, sc)
    exp = torch.nn.functional.linear(x.float(), ops.dequantize_fp8(qw, sc, torch.float32))
    # activation fp8 rounding dominates: relative error of a few percent of the row scale
    err = (got.float() - exp).abs().max() / exp.abs().max()
    assert float(err) < 0.08


@pytest.mark.parametrize("mode", [0, 1, 2, 3])
@pytest.mark.parametrize("m,width", [(1, 4096), (37, 8192), (300, 14336), (3, 28672),
                                     (2, 40960)])  # 40960: past the register-resident sizes
def test_quant_rows_fp8(mode, m, width):
    """Fused row-wise e4m3fn quantisation (norm / silu-mul / plain) vs the fp32 reference:
    scales match, codes dequantise to the reference values within e4m3 rounding."""
    torch.manual_seed(40 + mode)
    dt = torch.bfloat16
    x = torch.randn(m, 2 * width if mode == 1 else width, dtype=dt, device="cuda") * 3
    x[0] = 0 if mode == 2 else x[0]  # an all-zero row must not divide by zero
    w = (1 + 0.1 * torch.randn(width, dtype=dt, device="cuda")) if mode in (0, 3) else None
    res = torch.randn(m, width, dtype=dt, device="cuda") if mode == 3 else None
    res_cpu = res.cpu() if res is not None else None
    q, s = ops.quant_rows_fp8(x, mode, w, 1e-5, res)
    qr, sr = ops.quant_rows_fp8(x.cpu(), mode, None if w is None else w.cpu(), 1e-5, res_cpu)
    if mode == 3:  # residual stream updated in place, rounded like the bf16 add
        assert torch.equal(res.cpu(), res_cpu)
    close(s.cpu(), sr, 0.0, 2e-2)
    deq = q.view(torch.float8_e4m3fn).float().cpu() * s.cpu()
    ref_v = qr.view(torch.float8_e4m3fn).float() * sr
    # e4m3 has 3 mantissa bits: the reference rounds its normalised values to bf16 first,
    # so a value on a code boundary may land one code step (<= 1/8 relative) away
    err = (deq - ref_v).abs()
    assert bool((err <= 0.14 * ref_v.abs() + s.cpu()).all()), float(err.max())
    assert bool((deq.abs() <= 448 * s.cpu() * 1.0001).all())


@pytest.mark.parametrize("m", [1, 7, 64, 300])
def test_gemm_fp8_rowwise(m):
    """Row-wise-scaled fp8 GEMM (hipBLASLt via torch._scaled_mm) == fp32 GEMM of the
    dequantised operands."""
    torch.manual_seed(41)
    x = torch.randn(m, 4096, dtype=torch.bfloat16, device="cuda")
    w = torch.randn(1024, 4096, dtype=torch.bfloat16, device="cuda") * 0.05
    wq, ws = ops.quantize_fp8(w)
    xq, xs = ops.quant_rows_fp8(x)
    got = ops.gemm_fp8(xq, xs, wq, ws)
    exp = (xq.view(torch.float8_e4m3fn).float() * xs) @ \
        (wq.view(torch.float8_e4m3fn).float() * ws[:, None]).t()
    err = (got.float() - exp).abs().max() / exp.abs().max()
    assert float(err) < 1e-2


@pytest.mark.parametrize("nbytes", [16, 4096 + 48, 64 << 20])
def test_stream_read_probe(nbytes):
    """The HBM read probe (scripts/gpu/decode_sol.py) reads whole buffers of any 16-byte
    multiple, including a grid-stride remainder, and writes nothing."""
    x = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device="cuda")
    sink = torch.zeros(512, dtype=torch.int32, device="cuda")
    ops._native().stream_read(x, sink)
    torch.cuda.synchronize()
    assert bool((sink == 0).all())


@pytest.mark.parametrize("m", [1, 5, 16])
def test_fp8_decode_kernels_vs_fp32_reference(m):
    """the fp8 weight-only decode GEMVs against the fp32 PyTorch reference
    (ops/reference.py) of the same op on the dequantised weights - not against another
    kernel.  Plain projection, residual add, fused RMSNorm + gate_up + SiLU*up, fused
    RMSNorm + QKV + RoPE + paged K/V write."""
    torch.manual_seed(41)
    dt, H = torch.bfloat16, 2048
    x = torch.randn(m, H, dtype=dt, device="cuda")
    xf = x.float()

    def q(w, rowmap="plain"):
        qw, sc = ops.quantize_fp8(w)
        return ops.preshuffle_fp8(qw, rowmap), sc, ops.dequantize_fp8(qw, sc, torch.float32)

    w = torch.randn(1024, H, dtype=dt, device="cuda") * 0.05
    wq, sc, wf = q(w)
    exp = xf @ wf.t()
    close(ops.linear(x, wq, w_scale=sc), exp, 2e-2, 1e-2)
    res = torch.randn(m, 1024, dtype=dt, device="cuda")
    want = res.float() + exp
    ops.linear(x, wq, residual=res, w_scale=sc)
    close(res, want, 4e-2, 1e-2)
    eps, inter = 1e-5, 512
    ones = torch.ones(H, dtype=torch.float32, device="cuda")
    wg = torch.randn(2 * inter, H, dtype=dt, device="cuda") * 0.05
    gq, gs, gf = q(wg, "silu")
    exp = ref.silu_and_mul(ref.rms_norm(xf, ones, eps) @ gf.t())
    close(ops.decode_gate_up_silu(x, gq, eps, w_scale=gs), exp, 3e-2, 3e-2)
    hq, hkv, bs, nb = 8, 2, 16, 8
    wqkv = torch.randn((hq + 2 * hkv) * 128, H, dtype=dt, device="cuda") * 0.05
    kq, ks, kf = q(wqkv, "qkv")
    kc = torch.zeros(nb, hkv, bs, 128, dtype=dt, device="cuda")
    vc = torch.zeros(nb, hkv, 128, bs, dtype=dt, device="cuda")
    kc_r = torch.zeros(nb, hkv, bs, 128, dtype=torch.float32, device="cuda")
    vc_r = torch.zeros(nb, hkv, 128, bs, dtype=torch.float32, device="cuda")
    pos = torch.arange(3, 3 + m, dtype=torch.int32, device="cuda")
    slots = torch.arange(m, dtype=torch.int32, device="cuda") * 3
    cs = ref.rope_cos_sin(128, 64, 500000.0, None, device="cuda")
    got = ops.decode_qkv_rope(x, kq, eps, pos, slots, cs, kc, vc, hq, hkv, w_scale=ks)
    qkv = ref.rms_norm(xf, ones, eps) @ kf.t()
    exp = ref.rope_cache(qkv, pos, slots, cs, kc_r, vc_r, hq, hkv, 128)
    close(got, exp, 3e-2, 3e-2)
    close(kc, kc_r, 3e-2, 3e-2)
    close(vc, vc_r, 3e-2, 3e-2)


@pytest.mark.parametrize("m", [1, 5, 16, 17, 32])
def test_decode_gate_up_silu_8b_shape(m):
    """gate_up + SiLU at the Llama-3.1-8B decode shape (inter 14336, K 4096, pre-shuffled,
    1792 16-row tiles) vs fp32.  m 17 / 32: two MFMA row blocks at ops.DECODE_WAVES_MT2's wave count (small-prefill path)."""
    torch.manual_seed(m)
    dt = torch.bfloat16
    inter, H = 14336, 4096
    x = torch.randn(m, H, dtype=dt, device="cuda")
    wg = torch.randn(2 * inter, H, dtype=dt, device="cuda") * 0.02
    exp = ref.silu_and_mul(torch.nn.functional.linear(_norm_ref(x).float(), wg.float()))
    got = ops.decode_gate_up_silu(x, ops.preshuffle(wg, "silu"), 1e-5, preshuffled=True)
    close(got, exp.to(dt), 4e-2, 4e-2)
