"""Decode-path microbenchmarks on MI355X.

1. Skinny GEMM variants (waves x unroll x load policy) vs hipBLASLt (F.linear) at the
   Llama-3-8B decode shapes; reports us and effective weight-stream GB/s.
2. Decode attention: v1 (separate combine kernel) vs v2 (in-kernel combine) at the
   contexts of the fan-out workload.
Timings are medians of CUDA-event-timed loops over rotating weight copies totalling >= 768 MB
(three times the 256 MiB Infinity Cache), so weights are never MALL resident between calls -
the state they are in during a real decode step (15 GB of weights per step)."""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402

SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
          ("down", 4096, 14336), ("lm_head", 128256, 4096)]
VARIANTS = {0: "w8u4-nt", 1: "w8u8", 2: "w4u4", 3: "w4u8", 4: "w8u4", 5: "w16u4",
            6: "w8u2", 7: "w16u2", 8: "w8u2-ps", 9: "w16u2-ps", 10: "w8u4-ps",
            11: "w16u4-ps", 12: "w4u4-ps", 13: "w4u8-ps"}
PRESHUFFLED = {8, 9, 10, 11, 12, 13}
SWEEP = os.environ.get("MB_VARIANTS")  # e.g. "6,7,8,9,10,11,12,13"


def timeit(fn, iters=40, reps=3):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1000)
    return statistics.median(res)


def gemm_sweep():
    print("== skinny GEMM (us / GB/s)")
    hdr = f"{'shape':>8} {'M':>3} {'blaslt':>13}" + "".join(
        f" {v:>15}" for k, v in VARIANTS.items() if not SWEEP or str(k) in SWEEP.split(","))
    print(hdr)
    for name, n, k in SHAPES:
        nbytes = n * k * 2
        ncopy = max(4, math.ceil(768e6 / nbytes))
        ws = [torch.randn(n, k, dtype=torch.bfloat16, device="cuda") * 0.02 for _ in range(ncopy)]
        wps = [ops.preshuffle(w) for w in ws]
        for m in (1, 5, 16):
            x = torch.randn(m, k, dtype=torch.bfloat16, device="cuda")
            out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
            i = [0]

            def blas():
                i[0] = (i[0] + 1) % ncopy
                torch.nn.functional.linear(x, ws[i[0]])

            tb = timeit(blas)
            row = f"{name:>8} {m:3d} {tb:7.1f}/{nbytes / tb / 1e3:5.0f}"
            for vid in VARIANTS:
                if SWEEP and str(vid) not in SWEEP.split(","):
                    continue
                def f(vid=vid):
                    i[0] = (i[0] + 1) % ncopy
                    src = wps if vid in PRESHUFFLED else ws
                    torch.ops.atta.skinny_variant(out, x, src[i[0]], vid)
                try:
                    t = timeit(f)
                    row += f" {t:7.1f}/{nbytes / t / 1e3:5.0f}  "
                except RuntimeError:
                    row += f" {'n/a':>15}"
            print(row, flush=True)


def fp8_sweep():
    """Production GEMV path (ops.linear): pre-shuffled bf16 vs fp8 weights, cold caches."""
    print("== decode GEMV: bf16-ps vs fp8 (us / weight GB/s), waves 8 and 16")
    print(f"{'shape':>8} {'M':>3} {'bf16 w8':>13} {'bf16 w16':>13} {'fp8 w8':>13} {'fp8 w16':>13}")
    for name, n, k in SHAPES:
        nb16 = n * k * 2
        ncopy = max(4, math.ceil(768e6 / nb16))
        ws = [ops.preshuffle(torch.randn(n, k, dtype=torch.bfloat16, device="cuda") * 0.02)
              for _ in range(ncopy)]
        qs = []
        for w in ws:
            q, sc = ops.quantize_fp8(w)  # layout irrelevant for timing
            qs.append((ops.preshuffle_fp8(q), sc))
        for m in (1, 5):
            x = torch.randn(m, k, dtype=torch.bfloat16, device="cuda")
            out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
            row = f"{name:>8} {m:3d}"
            for fp8 in (False, True):
                for waves in (8, 16):
                    i = [0]

                    def f(fp8=fp8, waves=waves):
                        i[0] = (i[0] + 1) % ncopy
                        if fp8:
                            ops.linear(x, qs[i[0]][0], out=out, waves=waves, w_scale=qs[i[0]][1])
                        else:
                            ops.linear(x, ws[i[0]], out=out, waves=waves, preshuffled=True)
                    t = timeit(f)
                    nbytes = nb16 // 2 if fp8 else nb16
                    row += f" {t:7.1f}/{nbytes / t / 1e3:5.0f}"
            print(row, flush=True)
        del ws, qs
        torch.cuda.empty_cache()


def attn_sweep():
    print("== decode attention (us): v1 = kernel + combine, v2 = in-kernel combine")
    hq, hkv, bs = 32, 8, 16
    for B, ctx in ((1, 300), (1, 600), (5, 500), (5, 1000), (1, 3800), (12, 2000)):
        nblk = math.ceil(ctx / bs)
        nb = B * nblk + 8
        k = torch.randn(nb, hkv, bs, 128, dtype=torch.bfloat16, device="cuda")
        v = torch.randn(nb, hkv, 128, bs, dtype=torch.bfloat16, device="cuda")
        bt = torch.randperm(nb, device="cuda")[:B * nblk].view(B, nblk).to(torch.int32)
        kvlen = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        qstart = torch.arange(B + 1, dtype=torch.int32, device="cuda")
        q = torch.randn(B, hq, 128, dtype=torch.bfloat16, device="cuda")
        out = torch.empty_like(q)
        row = f"B={B:2d} ctx={ctx:5d}"
        for pt in (128, 256, 512):
            mp = math.ceil(4096 / pt)
            po = torch.empty(B * hkv * mp * 16 * 128, device="cuda")
            pl = torch.empty(B * hkv * mp * 16, device="cuda")
            cnt = torch.zeros(B * hkv, dtype=torch.int32, device="cuda")
            t1 = timeit(lambda: ops.attention_decode(q, k, v, bt, kvlen, qstart, 0.088, po, pl,
                                                     math.ceil(ctx / pt), pt, out=out))
            t2 = timeit(lambda: ops.attention_decode_v2(q, k, v, bt, kvlen, qstart, 0.088, po, pl,
                                                        cnt, mp, pt, out=out))
            row += f" | pt={pt}: v1 {t1:6.1f} v2 {t2:6.1f}"
        kv_bytes = B * ctx * hkv * 128 * 2 * 2
        row += f" | ideal@6TB/s {kv_bytes / 6e6:5.1f}"
        print(row, flush=True)


def grid_sweep():
    """Does the launch grid (empty partition workgroups) cost decode attention time?"""
    print("== decode attention v2 (us) vs grid z = max_parts (256-token partitions)")
    hq, hkv, bs = 32, 8, 16
    for B, ctx in ((1, 300), (5, 500), (5, 1000), (8, 1000), (5, 2000)):
        nblk = math.ceil(ctx / bs)
        nb = B * nblk + 8
        k = torch.randn(nb, hkv, bs, 128, dtype=torch.bfloat16, device="cuda")
        v = torch.randn(nb, hkv, 128, bs, dtype=torch.bfloat16, device="cuda")
        bt = torch.randperm(nb, device="cuda")[:B * nblk].view(B, nblk).to(torch.int32)
        kvlen = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
        qstart = torch.arange(B + 1, dtype=torch.int32, device="cuda")
        q = torch.randn(B, hq, 128, dtype=torch.bfloat16, device="cuda")
        out = torch.empty_like(q)
        need = math.ceil(ctx / 256)
        row = f"B={B:2d} ctx={ctx:5d} need={need:2d} |"
        for mp in (need, 16, 64):
            po = torch.empty(B * hkv * mp * 16 * 128, device="cuda")
            pl = torch.empty(B * hkv * mp * 16, device="cuda")
            cnt = torch.zeros(B * hkv, dtype=torch.int32, device="cuda")
            t = timeit(lambda: ops.attention_decode_v2(q, k, v, bt, kvlen, qstart, 0.088, po, pl,
                                                       cnt, mp, 256, out=out))
            row += f" mp={mp:2d}: {t:6.1f}"
        # padded batch: 8 extra dummy rows (kvlen 0) like a graph bucket
        print(row, flush=True)


if __name__ == "__main__":
    assert ops.native_available()
    what = sys.argv[1] if len(sys.argv) > 1 else "all"
    if what in ("all", "gemm"):
        gemm_sweep()
    if what in ("all", "attn"):
        attn_sweep()
    if what in ("all", "fp8"):
        fp8_sweep()
    if what in ("all", "grid"):
        grid_sweep()
