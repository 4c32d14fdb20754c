#!/usr/bin/env python3
"""A/B of the hand-written CDNA4 prefill GEMM (ops.prefill_gemm) against hipBLASLt
(torch F.linear / addmm) on the Llama-3.1-8B prefill projections, cold weights (4 rotating
copies so every call streams W from HBM, as in a real prefill), uniform random operands.

Reports per shape: us per call and dense TF/s (2*M*N*K; the SILU row counts both gate and up
columns).  The gate_up rows compare the fused SiLU-mul GEMM against hipBLASLt gate_up +
the silu_and_mul kernel (what the prefill path runs without it).

    python scripts/gpu/bench_prefill_gemm.py --m 512 1300 2600 > profiles/r3_prefill_gemm_ab.txt
    python scripts/gpu/bench_prefill_gemm.py --m 73 382 --bm 64 128 256 \
        --schedules hybrid splitk        # tile-height x schedule sweep, interleaved rounds
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402

SHAPES = {  # name: (N rows of W, K, mode)
    "qkv": (6144, 4096, ops.GEMM_PLAIN),
    "o+res": (4096, 4096, ops.GEMM_RESADD),
    "gate_up+silu": (28672, 4096, ops.GEMM_SILU),
    "down+res": (4096, 14336, ops.GEMM_RESADD),
}


def timed(fn, iters):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(0)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[512, 1300, 2600])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--only", default="")
    ap.add_argument("--fp8", action="store_true",
                    help="e4m3fn operands with row scales: ours vs hipBLASLt torch._scaled_mm")
    ap.add_argument("--schedule", default="hybrid", choices=["hybrid", "streamk", "dp", "splitk"])
    ap.add_argument("--group-m", type=int, default=4)
    ap.add_argument("--bm", type=int, nargs="+", default=[0],
                    help="tile heights to sweep (0 = the library's pick)")
    ap.add_argument("--schedules", nargs="+", default=None,
                    help="schedules to sweep per call (default: --schedule)")
    ap.add_argument("--rounds", type=int, default=3,
                    help="interleaved rounds of all variants; the median is reported")
    ap.add_argument("--tuned", default="",
                    help="TunableOp table for the hipBLASLt arm (agentic_traffic_testing_amd/"
                         "tuning; 'auto' = the shipped llama-3.1-8b table)")
    args = ap.parse_args()
    scheds = args.schedules or [args.schedule]
    if args.tuned:
        from agentic_traffic_testing_amd import tuning

        print(f"# library arm on the tuned table: {tuning.load(args.tuned, 'llama-3.1-8b')}")
    ops.prefill_gemm_config(args.schedule, args.group_m)
    dev = "cuda"
    print(f"# prefill GEMM A/B ({'fp8 e4m3fn, row scales' if args.fp8 else 'bf16'}), "
          f"{torch.cuda.get_device_name()}, cold weights x{args.copies}, random operands; "
          f"TF/s = 2*M*N*K / t; schedule {args.schedule}, group_m {args.group_m}; "
          f"stream-K error word checked at the end")
    for name, (n, k, mode) in SHAPES.items():
        if args.only and args.only not in name:
            continue
        # enough copies that the rotation (>= 768 MB) never fits the 256 MB Infinity Cache
        copies = max(args.copies, int(768e6 / (n * k * 2)) + 1)
        ws = [(torch.rand(n, k, device=dev) * 2 - 1).to(torch.bfloat16) / k ** 0.5
              for _ in range(copies)]
        if args.fp8:
            qs = [ops.quant_rows_fp8(w) for w in ws]
            ws = [q for q, _ in qs]
            wsc = [s.reshape(-1).contiguous() for _, s in qs]
        for m in args.m:
            x = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
            if args.fp8:
                x, xs = ops.quant_rows_fp8(x)
            nout = n // 2 if mode == ops.GEMM_SILU else n
            res = torch.randn(m, nout, device=dev).to(torch.bfloat16)
            out = torch.empty(m, nout, device=dev, dtype=torch.bfloat16)
            flops = 2.0 * m * n * k

            def make(bm, sched):
                def ours(i):
                    w = ws[i % len(ws)]
                    kw = dict(xs=xs, ws=wsc[i % len(ws)]) if args.fp8 else {}
                    if mode == ops.GEMM_RESADD:
                        ops.prefill_gemm(x, w, mode, residual=res, schedule=sched, bm=bm, **kw)
                    else:
                        ops.prefill_gemm(x, w, mode, out=out, schedule=sched, bm=bm, **kw)
                return ours

            def lin(i):
                w = ws[i % len(ws)]
                if args.fp8:
                    return ops.gemm_fp8(x, xs, w, wsc[i % len(ws)])
                return torch.nn.functional.linear(x, w)

            def blas(i):
                if mode == ops.GEMM_RESADD:
                    if args.fp8:
                        res.add_(lin(i))
                    else:
                        res.addmm_(x, ws[i % len(ws)].t())
                elif mode == ops.GEMM_SILU:
                    ops.silu_and_mul(lin(i))
                else:
                    lin(i)

            # numerics spot check against hipBLASLt (fp32 accumulate both), every variant
            ref = lin(0).float()
            if mode == ops.GEMM_SILU:
                ref = torch.nn.functional.silu(ref[:, :nout]) * ref[:, nout:]
            variants = [(bm, sc) for bm in args.bm for sc in scheds]
            err = 0.0
            for bm, sc in variants:
                kw = dict(xs=xs, ws=wsc[0]) if args.fp8 else {}
                got = ops.prefill_gemm(x, ws[0], mode if mode == ops.GEMM_SILU else 0,
                                       schedule=sc, bm=bm, **kw).float()
                err = max(err, ((got - ref).abs().max() / ref.abs().max()).item())
            times = {v: [] for v in variants}
            tb = []
            for _ in range(args.rounds):
                tb.append(timed(blas, args.iters))
                for v in variants:
                    times[v].append(timed(make(*v), args.iters))
            t_blas = sorted(tb)[len(tb) // 2]
            med = {v: sorted(t)[len(t) // 2] for v, t in times.items()}
            best = min(med, key=med.get)
            cols = " ".join(f"{bm or 'auto'}/{sc}:{med[(bm, sc)]:7.1f}" for bm, sc in variants)
            print(f"{name:13s} M={m:5d} N={n:6d} K={k:6d} | hipBLASLt {t_blas:8.1f} us "
                  f"{flops / t_blas / 1e6:6.0f} TF | {cols} | best {best[0] or 'auto'}/{best[1]} "
                  f"{med[best]:7.1f} us {flops / med[best] / 1e6:6.0f} TF "
                  f"{t_blas / med[best]:5.2f}x | rel err {err:.2e}", flush=True)
        del ws
    assert ops.prefill_gemm_error() == 0, "a cross-workgroup wait timed out"


if __name__ == "__main__":
    main()
