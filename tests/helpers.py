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
