"""Decode attention + o_proj pairs (Llama-3.1-8B shapes, B = 1 / 5, 3k context) with and
without the o_proj L2 prefetch workgroups of the attention launch (ops.oproj_prefetch_spec).
32 distinct o weights (1 GB, larger than the Infinity Cache) so every layer's o_proj is cold
unless the prefetch warmed it.  Prints us per (attention + o_proj) layer and per kernel."""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402


def ev_time(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) * 1000)
    return statistics.median(res)


def main():
    torch.manual_seed(0)
    dt, bs, hq, hkv, D, L = torch.bfloat16, 16, 32, 8, 128, 32
    H = hq * D
    ws = [ops.preshuffle(torch.randn(H, H, dtype=dt, device="cuda") * 0.02) for _ in range(L)]
    sink = torch.zeros(4, dtype=torch.int32, device="cuda")
    for B, ctx in ((1, 3000), (5, 1200), (5, 3000)):
        nblk = math.ceil(ctx / bs)
        k = torch.randn(B * nblk + 8, hkv, bs, D, dtype=dt, device="cuda")
        v = torch.randn(B * nblk + 8, hkv, D, bs, dtype=dt, device="cuda")
        bt = torch.arange(B * nblk, dtype=torch.int32, device="cuda").view(B, nblk)
        kvlen = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        qstart = torch.arange(B + 1, dtype=torch.int32, device="cuda")
        q = torch.randn(B, hq, D, dtype=dt, device="cuda")
        max_parts = 32
        po = torch.empty(B * hkv * max_parts * 16 * D, device="cuda")
        pl = torch.empty(B * hkv * max_parts * 16, device="cuda")
        cnt = torch.zeros(B * hkv, dtype=torch.int32, device="cuda")
        out = torch.empty_like(q)
        res = torch.randn(B, H, dtype=dt, device="cuda")
        waves = ops.decode_waves("o", True)
        scale = 1 / math.sqrt(D)

        def attn(li, chunks):
            pf = ops.oproj_prefetch_spec(ws[li], H, waves, B, hkv, sink, chunks=chunks)
            ops.attention_decode_v2(q, k, v, bt, kvlen, qstart, scale, po, pl, cnt,
                                    max_parts, 128, out=out, prefetch=pf)

        def oproj(li):
            ops.linear(out.view(B, H), ws[li], residual=res, waves=waves, preshuffled=True,
                       ksplit=None, proj="o")

        row = f"B={B} ctx={ctx}:"
        base_o = ev_time(lambda: [oproj(li) for li in range(L)]) / L
        row += f" o alone {base_o:6.2f}"
        for chunks in (0, 1, 2, 3, 4):
            a = ev_time(lambda: [attn(li, chunks) for li in range(L)]) / L
            ao = ev_time(lambda: [(attn(li, chunks), oproj(li)) for li in range(L)]) / L
            row += f" | pf{chunks}: attn {a:6.2f} attn+o {ao:6.2f}"
        print(row, flush=True)
        assert int(sink.abs().sum()) == 0


if __name__ == "__main__":
    main()
