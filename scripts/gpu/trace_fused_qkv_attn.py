"""Per-workgroup timeline of the fused qkv + decode-attention launch on MI355X.

Llama-3.1-8B decode shapes (qkv 6144 x 4096, Hq 32 / Hkv 8), ~3k-token contexts, 32
partitions (max_model_len 8192).  Times the fused launch against qkv + attention as two
launches (CUDA events, rotating cold weight copies), then runs the fused launch once with
``wg_trace`` and prints where the time goes: when the qkv tiles end, when the attention
workgroups start, get past their wait and end (100 MHz wall clock, 10 ns ticks).
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


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else float("nan")


def run(ctxs, dt=torch.bfloat16):
    B = len(ctxs)
    kvlens = [c + 1 if c > 0 else 0 for c in ctxs]
    nblk = [max(1, math.ceil(kv / BS)) for kv in kvlens]
    nb = sum(nblk) + 8
    perm = torch.randperm(nb)
    bt = torch.zeros(B, MAXP * 256 // BS, dtype=torch.int32)
    o = 0
    for i, n in enumerate(nblk):
        bt[i, :n] = perm[o:o + n].to(torch.int32)
        o += n
    bt = bt.cuda()
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
    ws = {"part_out": torch.empty(B * HKV * MAXP * 16 * 128, device="cuda"),
          "part_lse": torch.empty(B * HKV * MAXP * 16, device="cuda"),
          "counters": torch.zeros(B * HKV, dtype=torch.int32, device="cuda"),
          "side_kv": torch.zeros(B, HKV, 2, 128, dtype=dt, device="cuda"),
          "pub_counters": torch.zeros(HKV, dtype=torch.int32, device="cuda"),
          "exit_counters": torch.zeros(HKV, dtype=torch.int32, device="cuda"),
          "fused_error": torch.zeros(1, dtype=torch.int32, device="cuda"),
          "max_parts": MAXP}
    q = torch.empty(B, HQ, 128, dtype=dt, device="cuda")
    a = torch.empty(B, HQ, 128, dtype=dt, device="cuda")
    i = [0]

    def sep():
        i[0] = (i[0] + 1) % ncopy
        ops.decode_qkv_rope(x, ws_[i[0]], 1e-5, pos, slots, cs, k, v, HQ, HKV, q_out=q,
                            preshuffled=True)
        ops.attention_decode_v2(q, k, v, bt, kvlen, qstart, scale, ws["part_out"],
                                ws["part_lse"], ws["counters"], MAXP, 256, out=a, num_seqs=B)

    def qkv_only():
        i[0] = (i[0] + 1) % ncopy
        ops.decode_qkv_rope(x, ws_[i[0]], 1e-5, pos, slots, cs, k, v, HQ, HKV, q_out=q,
                            preshuffled=True)

    def attn_only():
        ops.attention_decode_v2(q, k, v, bt, kvlen, qstart, scale, ws["part_out"],
                                ws["part_lse"], ws["counters"], MAXP, 256, out=a, num_seqs=B)

    def fused(trace=None):
        i[0] = (i[0] + 1) % ncopy
        ops.decode_qkv_attention(x, ws_[i[0]], 1e-5, pos, slots, cs, k, v, HQ, HKV, bt, kvlen,
                                 scale, ws, q, a, wg_trace=trace)

    print(f"== B={B} ctx={ctxs}")
    print(f"  separate qkv+attn {timeit(sep):7.2f} us   (qkv {timeit(qkv_only):6.2f}, "
          f"attn {timeit(attn_only):6.2f})")
    print(f"  fused             {timeit(fused):7.2f} us", flush=True)
    # standalone attention timeline
    qkv_only()
    atr = torch.zeros(4 * B * HKV * MAXP, dtype=torch.int64, device="cuda")
    ops.set_attention_trace(atr)
    for _ in range(3):
        attn_only()
    torch.cuda.synchronize()
    ops.set_attention_trace(None)
    t = atr.view(MAXP, HKV, B, 4).cpu()  # grid (seqs, heads, parts): x fastest
    real = [(s_, h, p_) for s_ in range(B) for h in range(HKV)
            for p_ in range(math.ceil(kvlens[s_] / 256))]
    if real:
        t0a = min(int(t[p_, h, s_, 0]) for s_, h, p_ in real)
        col = lambda j: sorted((int(t[p_, h, s_, j]) - t0a) / 100.0 for s_, h, p_ in real)  # noqa
        for j, name in enumerate(("past RT1", "computed", "published", "end")):
            c = col(j)
            print(f"  attn {name:9s} p0/p50/max {c[0]:6.2f} {c[len(c) // 2]:6.2f} {c[-1]:6.2f}")
    kv_real = kvlen.clone()
    kvlen.zero_()  # no attention work: the qkv tiles alone inside the fused launch
    print(f"  fused, kvlen 0    {timeit(fused):7.2f} us", flush=True)
    kvlen.copy_(kv_real)
    n_tiles = (HQ + 2 * HKV) * 8
    nwg = n_tiles + B * HKV * MAXP
    tr = torch.zeros(4 * nwg, dtype=torch.int64, device="cuda")
    for _ in range(3):
        fused(tr)
    torch.cuda.synchronize()
    assert int(ws["fused_error"][0]) == 0
    t = tr.view(nwg, 4).cpu()
    t0 = int(t[:, 0].min())
    us = lambda c: ((c - t0).double() / 100.0).tolist()  # noqa: E731  (10 ns ticks -> us)
    st, wt, en = us(t[:, 0]), us(t[:, 1]), us(t[:, 2])
    qkv = range(n_tiles)
    real = [n_tiles + (s * HKV + h) * MAXP + p for s in range(B) for h in range(HKV)
            for p in range(math.ceil(kvlens[s] / 256))]
    empty = sorted(set(range(n_tiles, nwg)) - set(real))
    print(f"  kernel span {max(en) - min(st):7.2f} us; qkv tiles {n_tiles}, real attention WGs "
          f"{len(real)}, empty {len(empty)}")
    print(f"  qkv   start p0/p50/max {pct([st[j] for j in qkv], 0):6.2f} "
          f"{pct([st[j] for j in qkv], .5):6.2f} {max(st[j] for j in qkv):6.2f}   end p50/p90/max "
          f"{pct([en[j] for j in qkv], .5):6.2f} {pct([en[j] for j in qkv], .9):6.2f} "
          f"{max(en[j] for j in qkv):6.2f}")
    print(f"  attn  start p0/p50/max {pct([st[j] for j in real], 0):6.2f} "
          f"{pct([st[j] for j in real], .5):6.2f} {max(st[j] for j in real):6.2f}   past-wait "
          f"p50/max {pct([wt[j] for j in real], .5):6.2f} {max(wt[j] for j in real):6.2f}   end "
          f"p50/max {pct([en[j] for j in real], .5):6.2f} {max(en[j] for j in real):6.2f}")
    if empty:
        print(f"  empty start p50/max {pct([st[j] for j in empty], .5):6.2f} "
              f"{max(st[j] for j in empty):6.2f}   end max {max(en[j] for j in empty):6.2f}")
    cus = len(set(t[:n_tiles, 3].tolist()))
    print(f"  distinct CU ids among qkv tiles: {cus}", flush=True)


def producers_only():
    """ATTA_FUSED_PRODUCERS_ONLY=1: the fused launch with its qkv tiles only (timing)."""
    B, dt, ncopy = 1, torch.bfloat16, 8
    x = torch.randn(B, H, dtype=dt, device="cuda")
    ws_ = [ops.preshuffle(torch.randn((HQ + 2 * HKV) * 128, H, dtype=dt, device="cuda") * 0.02,
                          "qkv") for _ in range(ncopy)]
    cs = ref.rope_cos_sin(128, 8192, 500000.0, None, device="cuda")
    k = torch.zeros(64, HKV, BS, 128, dtype=dt, device="cuda")
    v = torch.zeros(64, HKV, 128, BS, dtype=dt, device="cuda")
    bt = torch.zeros(B, 16, dtype=torch.int32, device="cuda")
    kvlen = torch.zeros(B, dtype=torch.int32, device="cuda")
    pos = torch.zeros(B, dtype=torch.int32, device="cuda")
    slots = torch.full((B,), -1, dtype=torch.int32, device="cuda")
    ws = {"part_out": torch.empty(B * HKV * MAXP * 16 * 128, device="cuda"),
          "part_lse": torch.empty(B * HKV * MAXP * 16, device="cuda"),
          "counters": torch.zeros(B * HKV, dtype=torch.int32, device="cuda"),
          "side_kv": torch.zeros(B, HKV, 2, 128, dtype=dt, device="cuda"),
          "pub_counters": torch.zeros(HKV, dtype=torch.int32, device="cuda"),
          "exit_counters": torch.zeros(HKV, dtype=torch.int32, device="cuda"),
          "fused_error": torch.zeros(1, dtype=torch.int32, device="cuda"),
          "max_parts": MAXP}
    q = torch.empty(B, HQ, 128, dtype=dt, device="cuda")
    a = torch.empty(B, HQ, 128, dtype=dt, device="cuda")
    i = [0]

    def sep():
        i[0] = (i[0] + 1) % ncopy
        ops.decode_qkv_rope(x, ws_[i[0]], 1e-5, pos, slots, cs, k, v, HQ, HKV, q_out=q,
                            preshuffled=True)

    def fused():
        i[0] = (i[0] + 1) % ncopy
        ops.decode_qkv_attention(x, ws_[i[0]], 1e-5, pos, slots, cs, k, v, HQ, HKV, bt, kvlen,
                                 1.0, ws, q, a)

    print(f"producers only: standalone qkv {timeit(sep):6.2f} us, fused-kernel qkv tiles "
          f"{timeit(fused):6.2f} us", flush=True)


if __name__ == "__main__":
    assert ops.native_available()
    if os.environ.get("ATTA_FUSED_PRODUCERS_ONLY"):
        producers_only()
        sys.exit(0)
    print(f"poll sleeps {os.environ.get('ATTA_FUSED_POLL_SLEEPS', '1')}")
    run([3000])
    if len(sys.argv) < 2:
        run([3000, 3100, 2900, 3050, 2950, 0, 0, 0])
