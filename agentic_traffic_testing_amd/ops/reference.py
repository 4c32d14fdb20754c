"""Plain-PyTorch (fp32 math) definitions of every native op.

These are (1) the numerics oracle the GPU tests compare the HIP kernels against and
(2) the implementation used when the engine runs on CPU tensors (the CPU test tier;
there is no GPU in the build container).  A GPU tensor never reaches this module through
``ops`` - the dispatch in ``ops/__init__.py`` is strictly by tensor device.

Semantics match ``ops/csrc/*.hip`` exactly, including where values are rounded to the
activation dtype.
"""
from __future__ import annotations

import math

import torch


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    n = (xf * inv).to(x.dtype)
    return (n.float() * w.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float):
    """Returns (normed, new_residual); new_residual = (x + residual) rounded to dtype."""
    r = (x.float() + residual.float()).to(x.dtype)
    return rms_norm(r, w, eps), r


def silu_and_mul(x: torch.Tensor) -> torch.Tensor:
    i = x.shape[-1] // 2
    g = x[..., :i].float()
    s = (g / (1.0 + torch.exp(-g))).to(x.dtype)
    return (s.float() * x[..., i:].float()).to(x.dtype)


def rope_rotate(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, H, D] -> rotated (neox rotate-half), fp32 math, rounded to x.dtype."""
    d = x.shape[-1]
    h = d // 2
    cs = cos_sin[positions.long()].float()  # [T, D]
    c = cs[:, None, :h]
    s = cs[:, None, h:]
    xf = x.float()
    x1, x2 = xf[..., :h], xf[..., h:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1).to(x.dtype)


def rope_cache(qkv, positions, slot_mapping, cos_sin, k_cache, v_cache, n_q_heads, n_kv_heads,
               head_dim):
    """Returns rotated q [T, Hq, D]; writes k (rotated) / v into the paged caches in place.

    k_cache [nb, Hkv, BS, D]; v_cache [nb, Hkv, D, BS] (transposed)."""
    t = qkv.shape[0]
    q = qkv[:, : n_q_heads * head_dim].reshape(t, n_q_heads, head_dim)
    k = qkv[:, n_q_heads * head_dim:(n_q_heads + n_kv_heads) * head_dim].reshape(t, n_kv_heads, head_dim)
    v = qkv[:, (n_q_heads + n_kv_heads) * head_dim:(n_q_heads + 2 * n_kv_heads) * head_dim].reshape(
        t, n_kv_heads, head_dim)
    qr = rope_rotate(q, positions, cos_sin)
    kr = rope_rotate(k, positions, cos_sin)
    bs = k_cache.shape[2]
    sm = slot_mapping.long()
    ok = sm >= 0
    if bool(ok.any()):
        s = sm[ok]
        page, off = s // bs, s % bs
        k_cache[page, :, off, :] = kr[ok].to(k_cache.dtype)
        v_cache[page, :, :, off] = v[ok].to(v_cache.dtype)
    return qr


def gather_kv(k_cache, v_cache, block_table_row, kvlen):
    """Materialise [kvlen, Hkv, D] K and V for one sequence from the paged cache."""
    bs = k_cache.shape[2]
    nblk = (kvlen + bs - 1) // bs
    pages = block_table_row[:nblk].long()
    k = k_cache[pages]  # [nblk, Hkv, BS, D]
    v = v_cache[pages]  # [nblk, Hkv, D, BS]
    k = k.permute(0, 2, 1, 3).reshape(nblk * bs, k.shape[1], k.shape[3])[:kvlen]
    v = v.permute(0, 3, 1, 2).reshape(nblk * bs, v.shape[1], v.shape[2])[:kvlen]
    return k, v


def paged_attention(q, k_cache, v_cache, block_tables, seq_kvlen, seq_qstart, scale, out=None):
    """Causal attention of every query token over its sequence's paged KV (fp32 math).

    q [Tq, Hq, D]; query token j of sequence s sits at position kvlen - qlen + j.
    Returns [Tq, Hq, D] in q.dtype.  With ``out`` given, only the rows of the listed
    sequences are written."""
    if out is None:
        out = torch.zeros_like(q)
    hq = q.shape[1]
    s_count = seq_kvlen.shape[0]
    for s in range(s_count):
        kvlen = int(seq_kvlen[s])
        q0, q1 = int(seq_qstart[s]), int(seq_qstart[s + 1])
        qlen = q1 - q0
        if qlen == 0 or kvlen == 0:
            continue
        k, v = gather_kv(k_cache, v_cache, block_tables[s], kvlen)
        hkv = k.shape[1]
        g = hq // hkv
        k = k.float().repeat_interleave(g, dim=1)  # [kv, Hq, D]
        v = v.float().repeat_interleave(g, dim=1)
        qs = q[q0:q1].float()  # [qlen, Hq, D]
        scores = torch.einsum("qhd,khd->hqk", qs, k) * scale
        qpos = torch.arange(kvlen - qlen, kvlen, device=q.device)[:, None]
        kpos = torch.arange(kvlen, device=q.device)[None, :]
        scores = scores.masked_fill((kpos > qpos)[None], float("-inf"))
        p = torch.softmax(scores, dim=-1)
        out[q0:q1] = torch.einsum("hqk,khd->qhd", p, v).to(q.dtype)
    return out


def _sample_scores(lf: torch.Tensor, r: int, temperature, seeds, steps, vocab_offset: int):
    t = float(temperature[r])
    if not t > 1e-5:
        return lf[r]
    idx = torch.arange(vocab_offset, vocab_offset + lf.shape[1], dtype=torch.int64)
    return lf[r] / t + gumbel_noise(int(seeds[r]), int(steps[r]), idx).to(lf.device)


def sample(logits: torch.Tensor, temperature: torch.Tensor, seeds: torch.Tensor,
           steps: torch.Tensor, vocab_offset: int = 0) -> torch.Tensor:
    """Greedy for temperature<=1e-5, else Gumbel-max with the kernel's counter-based RNG.
    ``vocab_offset`` = global id of column 0 (TP vocab shard); returned ids are global."""
    lf = logits.float()
    out = torch.empty(lf.shape[0], dtype=torch.long, device=logits.device)
    for r in range(lf.shape[0]):
        sc = _sample_scores(lf, r, temperature, seeds, steps, vocab_offset)
        out[r] = int(torch.argmax(sc)) + vocab_offset
    return out


def sample_topkp(logits: torch.Tensor, temperature, top_p, top_k, seeds,
                 steps) -> torch.Tensor:
    """top-k / top-p sampling with the kernel's definition (ops/csrc/sampling.hip): x =
    logit * (1/T) in fp32; keep x >= the k-th largest x (top_k in (0, vocab)); then keep x >=
    thr_p, the value at which the descending cumulative mass (32.32 fixed-point e^(x - max)
    over the kept set) first reaches ceil(p * Z) (top_p < 1); argmax of x + Gumbel over the
    kept set (lowest index on ties).  Greedy rows (T <= 1e-5) take argmax(logit)."""
    lf = logits.float().cpu()
    out = torch.empty(lf.shape[0], dtype=torch.long)
    V = lf.shape[1]
    for r in range(lf.shape[0]):
        t = float(temperature[r])
        if not t > 1e-5:
            out[r] = int(torch.argmax(lf[r]))
            continue
        inv_t = torch.tensor(1.0, dtype=torch.float32) / torch.tensor(t, dtype=torch.float32)
        x = lf[r] * inv_t
        keep = torch.ones(V, dtype=torch.bool)
        k = int(top_k[r])
        if 0 < k < V:
            keep &= x >= torch.topk(x, k).values[-1]
        p = float(top_p[r])
        if p < 1.0:
            w = torch.where(keep, torch.floor((torch.exp(x - x.max()).double()) * 2.0 ** 32),
                            torch.zeros((), dtype=torch.float64)).long()
            z = int(w.sum())
            target = max(1, math.ceil(float(torch.tensor(p, dtype=torch.float32)) * z))
            xs, order = torch.sort(torch.where(keep, x, torch.tensor(float("-inf"))),
                                   descending=True, stable=True)
            cum = torch.cumsum(w[order], 0)
            j = int(torch.nonzero(cum >= target)[0, 0])
            keep &= x >= xs[j]
        idx = torch.arange(V, dtype=torch.int64)
        sc = x + gumbel_noise(int(seeds[r]), int(steps[r]), idx)
        sc = torch.where(keep, sc, torch.tensor(float("-inf")))
        out[r] = int(torch.argmax(sc))
    return out.to(logits.device)


def _ordered_bits(v: float) -> int:
    import struct

    b = struct.unpack("<I", struct.pack("<f", v))[0]
    return (~b & 0xFFFFFFFF) if b & 0x80000000 else (b | 0x80000000)


def sample_keys(logits: torch.Tensor, temperature: torch.Tensor, seeds: torch.Tensor,
                steps: torch.Tensor, vocab_offset: int = 0) -> torch.Tensor:
    """Signed-orderable packed (score, -id) keys of each row's winner, as the kernel's
    ``finalize="key"`` mode emits them: MAX over TP shards picks the global winner."""
    lf = logits.float()
    out = torch.empty(lf.shape[0], dtype=torch.long, device=logits.device)
    for r in range(lf.shape[0]):
        sc = _sample_scores(lf, r, temperature, seeds, steps, vocab_offset)
        j = int(torch.argmax(sc))
        key = (_ordered_bits(float(sc[j])) << 32) | (0xFFFFFFFF - (j + vocab_offset))
        key ^= 1 << 63
        out[r] = key - (1 << 64) if key >= (1 << 63) else key
    return out


_M64 = (1 << 64) - 1


def _mix64_t(z: torch.Tensor) -> torch.Tensor:
    # splitmix64 finaliser on uint64 values held in int64 tensors (wrapping arithmetic)
    z = z + torch.tensor(0x9E3779B97F4A7C15 - (1 << 64), dtype=torch.int64)
    z = (z ^ _srl(z, 30)) * torch.tensor(0xBF58476D1CE4E5B9 - (1 << 64), dtype=torch.int64)
    z = (z ^ _srl(z, 27)) * torch.tensor(0x94D049BB133111EB - (1 << 64), dtype=torch.int64)
    return z ^ _srl(z, 31)


def _srl(z: torch.Tensor, n: int) -> torch.Tensor:
    """Logical right shift of int64-as-uint64."""
    return (z >> n) & ((1 << (64 - n)) - 1)


def _to_i64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


def gumbel_noise(seed: int, step: int, idx: torch.Tensor) -> torch.Tensor:
    inner = torch.tensor(_to_i64(step * 0x100000001B3), dtype=torch.int64) + idx
    h = _mix64_t(torch.tensor(_to_i64(seed), dtype=torch.int64) ^ _mix64_t(inner))
    u = (_srl(h, 40).double() + 0.5) * (1.0 / 16777216.0)
    return (-torch.log(-torch.log(u.float()))).float()


def rope_cos_sin(head_dim: int, max_pos: int, theta: float, scaling: dict | None = None,
                 device="cpu") -> torch.Tensor:
    """[max_pos, head_dim] fp32 table: cos in [:D/2], sin in [D/2:].  Implements llama3
    frequency scaling (factor / low_freq_factor / high_freq_factor / original_max_pos)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling.get("factor", 8.0)
        low = scaling.get("low_freq_factor", 1.0)
        high = scaling.get("high_freq_factor", 4.0)
        orig = scaling.get("original_max_position_embeddings", 8192)
        low_wl, high_wl = orig / low, orig / high
        wl = 2 * math.pi / inv
        smooth = (orig / wl - low) / (high - low)
        scaled = torch.where(wl > low_wl, inv / factor, inv)
        mid = (wl <= low_wl) & (wl >= high_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)
