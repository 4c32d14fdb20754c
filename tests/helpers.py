"""Shared test helpers: an independent dense (unpaged) Llama forward used as the oracle."""
import torch
import torch.nn.functional as F

from agentic_traffic_testing_amd.ops import reference as ref


@torch.no_grad()
def dense_logits(model, ids):
    """Full-sequence causal forward without paging / kernels; returns last-row logits."""
    c = model.cfg
    dev = model.embed.device
    x = F.embedding(torch.tensor(ids, device=dev), model.embed)
    T = len(ids)
    D = model.head_dim
    nq, nkv = model.n_heads, model.n_kv_heads
    pos = torch.arange(T, device=dev)
    mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=dev), 1)[None]
    for L in model.layers:
        h = ref.rms_norm(x, L.input_norm, c.rms_norm_eps)
        qkv = F.linear(h, L.qkv)
        q = qkv[:, :nq * D].view(T, nq, D)
        k = qkv[:, nq * D:(nq + nkv) * D].view(T, nkv, D)
        v = qkv[:, (nq + nkv) * D:(nq + 2 * nkv) * D].view(T, nkv, D)
        q = ref.rope_rotate(q, pos, model.cos_sin)
        k = ref.rope_rotate(k, pos, model.cos_sin)
        kk = k.float().repeat_interleave(model.g, 1)
        vv = v.float().repeat_interleave(model.g, 1)
        s = torch.einsum("qhd,khd->hqk", q.float(), kk) * model.scale
        s = s.masked_fill(mask, float("-inf"))
        a = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), vv).to(x.dtype)
        x = (x.float() + F.linear(a.reshape(T, -1), L.o).float()).to(x.dtype)
        h = ref.rms_norm(x, L.post_norm, c.rms_norm_eps)
        x = (x.float() + F.linear(ref.silu_and_mul(F.linear(h, L.gate_up)), L.down).float()).to(x.dtype)
    x = ref.rms_norm(x, model.norm, c.rms_norm_eps)
    return F.linear(x[-1:], model.lm_head)[0].float()


def greedy_reference(model, prompt, n):
    ids = list(prompt)
    out = []
    for _ in range(n):
        t = int(torch.argmax(dense_logits(model, ids)))
        out.append(t)
        ids.append(t)
    return out


def _qdq_rows(t, rows):
    """Per-token e4m3fn quantise -> dequantise of rows [0, rows) (ops.quant_rows_fp8 on the
    CPU, the prefill path's activation quantisation); later rows pass through."""
    from agentic_traffic_testing_amd import ops

    if rows <= 0:
        return t
    q, s = ops.quant_rows_fp8(t[:rows].float().cpu())
    deq = (q.view(torch.float8_e4m3fn).float() * s).to(t.device)
    return torch.cat([deq, t[rows:].float()], 0)


@torch.no_grad()
def dense_logits_fp8(model, ids, n_prompt):
    """fp32 oracle of an fp8 model (uint8 e4m3fn weights + per-row scales): every projection
    on the DEQUANTISED weights, in fp32.  The engine quantises the activations of prefill rows
    per token (quant_rows_fp8 fused into the norm / SiLU / attention-output producers, then an
    fp8 GEMM) while decode rows keep 16-bit activations (weight-only fp8 GEMVs), so rows
    [0, n_prompt) get the same quantise-dequantise here, later rows none."""
    from agentic_traffic_testing_amd import ops

    c = model.cfg
    dev = model.embed.device
    x = F.embedding(torch.tensor(ids, device=dev), model.embed).float()
    T = len(ids)
    D = model.head_dim
    nq, nkv = model.n_heads, model.n_kv_heads
    pos = torch.arange(T, device=dev)
    mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=dev), 1)[None]
    deq = lambda w, s: ops.dequantize_fp8(w, s, torch.float32)  # noqa: E731
    P = min(n_prompt, T)
    for L in model.layers:
        h = _qdq_rows(ref.rms_norm(x, L.input_norm.float(), c.rms_norm_eps), P)
        qkv = (h @ deq(L.qkv, L.qkv_s).t()).to(model.dtype).float()
        q = qkv[:, :nq * D].view(T, nq, D)
        k = qkv[:, nq * D:(nq + nkv) * D].view(T, nkv, D)
        v = qkv[:, (nq + nkv) * D:(nq + 2 * nkv) * D].view(T, nkv, D)
        q = ref.rope_rotate(q, pos, model.cos_sin)
        k = ref.rope_rotate(k, pos, model.cos_sin)
        kk = k.float().repeat_interleave(model.g, 1)
        vv = v.float().repeat_interleave(model.g, 1)
        s = torch.einsum("qhd,khd->hqk", q.float(), kk) * model.scale
        s = s.masked_fill(mask, float("-inf"))
        a = torch.einsum("hqk,khd->qhd", torch.softmax(s, -1), vv)
        a = _qdq_rows(a.reshape(T, -1).to(model.dtype).float(), P)
        x = (x + a @ deq(L.o, L.o_s).t()).to(model.dtype).float()
        h = _qdq_rows(ref.rms_norm(x, L.post_norm.float(), c.rms_norm_eps), P)
        gu = h @ deq(L.gate_up, L.gate_up_s).t()
        if getattr(model, "prefill_gemm", "") != "atta":
            gu = gu.to(model.dtype).float()
        else:  # the fused SiLU-mul GEMM epilogue: prefill rows see fp32 gate / up values
            gu = torch.cat([gu[:P], gu[P:].to(model.dtype).float()])
        g = ref.silu_and_mul(gu)
        g = _qdq_rows(g.to(model.dtype).float(), P)
        x = (x + g @ deq(L.down, L.down_s).t()).to(model.dtype).float()
    x = ref.rms_norm(x, model.norm.float(), c.rms_norm_eps)
    return (x[-1:] @ model.lm_head.float().t())[0]


def greedy_reference_fp8(model, prompt, n):
    ids = list(prompt)
    out = []
    for _ in range(n):
        t = int(torch.argmax(dense_logits_fp8(model, ids, len(prompt))))
        out.append(t)
        ids.append(t)
    return out
