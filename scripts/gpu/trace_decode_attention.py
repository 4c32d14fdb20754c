"""Per-workgroup timeline of the decode attention kernel on MI355X (ops.set_attention_trace).

Llama-3.1-8B decode shapes (Hq 32 / Hkv 8, head_dim 128), ~3k-token contexts, a 32-partition
grid (max_model_len 8192).  Times qkv + attention as two launches (CUDA events, rotating cold
weight copies), then records, for every workgroup that owns context: past round trip 1
(block table + lengths), partition computed, partial published (arrival counter), end - on
the 100 MHz wall clock.  The gaps show where a latency-bound split-K decode attention spends
its time (profiles/r2_fused_qkv_attn_wg_timeline.txt).
"""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402
from agentic_traffic_testing_amd.ops import reference as ref  # noqa: E402

HQ, HKV, H, BS, MAXP = 32, 8, 4096, 16, 32
PT = int(os.environ.get("PT", "256"))  # partition tokens (128 / 256 / 512)


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1000)
    return statistics.median(res)


def run(ctxs, dt=torch.bfloat16):
    B = len(ctxs)
    kvlens = [c + 1 if c > 0 else 0 for c in ctxs]
    nblk = [max(1, math.ceil(kv / BS)) for kv in kvlens]
    perm = torch.randperm(sum(nblk) + 8)
    bt = torch.zeros(B, MAXP * 512 // BS, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nblk):
        bt[i, :n] = perm[o:o + n].to(torch.int32)
        o += n
    bt = bt.cuda()
    nb = int(perm.numel())
    k = torch.randn(nb, HKV, BS, 128, dtype=dt, device="cuda")
    v = torch.randn(nb, HKV, 128, BS, dtype=dt, device="cuda")
    kvlen = torch.tensor(kvlens, dtype=torch.int32, device="cuda")
    qstart = torch.arange(B + 1, dtype=torch.int32, device="cuda")
    pos = torch.tensor([max(kv - 1, 0) for kv in kvlens], dtype=torch.int32, device="cuda")
    slots = torch.tensor([int(bt[i, (kv - 1) // BS]) * BS + (kv - 1) % BS if kv > 0 else -1
                          for i, kv in enumerate(kvlens)], dtype=torch.int32, device="cuda")
    x = torch.randn(B, H, dtype=dt, device="cuda")
    ncopy = 8  # 8 x 50 MB: beyond the 256 MB Infinity Cache
    ws_ = [ops.preshuffle(torch.randn((HQ + 2 * HKV) * 128, H, dtype=dt, device="cuda") * 0.02,
                          "qkv") for _ in range(ncopy)]
    cs = ref.rope_cos_sin(128, 8192, 500000.0, None, device="cuda")
    scale = 1 / math.sqrt(128)
    po = torch.empty(B * HKV * MAXP * 16 * 128, device="cuda")
    pl = torch.empty(B * HKV * MAXP * 16, device="cuda")
    cnt = torch.zeros(B * HKV, dtype=torch.int32, device="cuda")
    q = torch.empty(B, HQ, 128, dtype=dt, device="cuda")
    a = torch.empty(B, HQ, 128, dtype=dt, device="cuda")
    i = [0]

    def qkv_only():
        i[0] = (i[0] + 1) % ncopy
        ops.decode_qkv_rope(x, ws_[i[0]], 1e-5, pos, slots, cs, k, v, HQ, HKV, q_out=q,
                            preshuffled=True)

    def attn_only():
        ops.attention_decode_v2(q, k, v, bt, kvlen, qstart, scale, po, pl, cnt, MAXP, PT,
                                out=a, num_seqs=B)

    print(f"== B={B} ctx={ctxs} partition tokens {PT}")
    print(f"  qkv {timeit(qkv_only):6.2f} us, attention {timeit(attn_only):6.2f} us", flush=True)
    qkv_only()
    atr = torch.zeros(4 * B * HKV * MAXP, dtype=torch.int64, device="cuda")
    ops.set_attention_trace(atr)
    for _ in range(3):
        attn_only()
    torch.cuda.synchronize()
    ops.set_attention_trace(None)
    t = atr.view(MAXP, HKV, B, 4).cpu()  # grid (seqs, heads, parts): x fastest
    real = [(s_, h, p_) for s_ in range(B) for h in range(HKV)
            for p_ in range(math.ceil(kvlens[s_] / PT))]
    t0 = min(int(t[p_, h, s_, 0]) for s_, h, p_ in real)
    for j, name in enumerate(("past RT1", "computed", "published", "end")):
        c = sorted((int(t[p_, h, s_, j]) - t0) / 100.0 for s_, h, p_ in real)
        print(f"  {name:9s} p0/p50/max {c[0]:6.2f} {c[len(c) // 2]:6.2f} {c[-1]:6.2f} us",
              flush=True)


if __name__ == "__main__":
    assert ops.native_available()
    # CTXS="300;300,300,300,300,300" picks the batches (';' between batches, ',' inside one)
    spec = os.environ.get("CTXS")
    if spec:
        for b in spec.split(";"):
            run([int(c) for c in b.split(",")])
    else:
        run([3000])
        run([3000, 3100, 2900, 3050, 2950, 0, 0, 0])
