#!/usr/bin/env python3
"""Probe: small-M prefill GEMMs (the fan-out burst, M = 400-512) as hipBLASLt split-K
through a strided-batched GEMM (x[:, ks] @ W[:, ks].T for S K-slices, then a sum over the
slices) vs one F.linear.  hipBLASLt's own pick at M = 400 for down (N 4096, K 14336) runs at
~0.5 PF/s (profiles/r3_prefill400_summary.txt): 2 x 16 output tiles of 256 x 256 leave most CUs
idle unless K is split.

Cold weights (4 rotating copies), us per call.  out_dtype=float32 partials where the build
supports it (bf16 partials otherwise, reported).
"""
from __future__ import annotations

import argparse

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
          "down": (4096, 14336)}


def timed(fn, iters=20):
    torch.cuda.synchronize()
    fn(0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(iters):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[400, 512])
    ap.add_argument("--rocblas", action="store_true", help="also time rocBLAS (no split-K)")
    ap.add_argument("--no-split", action="store_true")
    a = ap.parse_args()
    dev = "cuda"
    try:
        t = torch.randn(2, 8, 64, device=dev, dtype=torch.bfloat16)
        torch.bmm(t, t.transpose(1, 2), out_dtype=torch.float32)
        f32 = True
    except Exception as e:  # noqa: BLE001
        print(f"# bmm out_dtype=float32 unavailable ({type(e).__name__}); bf16 partials")
        f32 = False
    print(f"# split-K via strided-batched hipBLASLt, {torch.cuda.get_device_name()}, cold W x4")
    for m in a.m:
        for name, (n, k) in SHAPES.items():
            ws = [torch.randn(n, k, device=dev, dtype=torch.bfloat16) / 64 for _ in range(4)]
            x = torch.randn(m, k, device=dev, dtype=torch.bfloat16)
            ref = (x.float() @ ws[0].float().t())
            base = timed(lambda i: F.linear(x, ws[i % 4]))
            row = f"{name:8s} M={m:4d} N={n:5d} K={k:5d} | linear {base:7.1f} us"
            if a.rocblas:
                torch.backends.cuda.preferred_blas_library("cublas")  # = rocBLAS on ROCm
                rb = timed(lambda i: F.linear(x, ws[i % 4]))
                torch.backends.cuda.preferred_blas_library("cublaslt")
                row += f" | rocBLAS {rb:7.1f} us (x{base / rb:4.2f})"
            for s in (() if a.no_split else (2, 4, 8)):
                if k % (s * 64):
                    continue
                ks = k // s

                def run(i, s=s, ks=ks):
                    w = ws[i % 4]
                    xs = x.view(m, s, ks).transpose(0, 1)
                    wt = w.view(n, s, ks).transpose(0, 1).transpose(1, 2)
                    if f32:
                        part = torch.bmm(xs, wt, out_dtype=torch.float32)
                    else:
                        part = torch.bmm(xs, wt)
                    return part.sum(0, dtype=torch.float32).to(torch.bfloat16)

                t = timed(run)
                err = ((run(0).float() - ref).abs().max() / ref.abs().max()).item()
                row += f" | S={s} {t:7.1f} us (x{base / t:4.2f}, err {err:.1e})"
            print(row, flush=True)
            del ws


if __name__ == "__main__":
    main()
