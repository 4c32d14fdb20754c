#!/usr/bin/env python3
"""Does warming a decode weight into the Infinity Cache (MALL) before its GEMV pay?

For each Llama-3.1-8B decode projection (pre-shuffled bf16, M = 5, production skinny GEMV):
  cold   - rotating weight copies totalling >= 768 MB (3x the MALL): every call streams HBM
  warm   - loop [read(W_i); gemv(W_i)]: a separate read kernel touched W just before
  other  - loop [read(W_i+1); gemv(W_i)]: the same read traffic, the GEMV's weight cold
  (warm - other) per call = what a prefetch of W into the MALL saves the GEMV.

    python scripts/gpu/probe_mall.py > profiles/r3_probe_mall.txt
"""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402

SHAPES = [("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336)]


def timeit(fn, iters=24, reps=3):
    for _ in range(4):
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


def main():
    print(f"# MALL warm-up probe, {torch.cuda.get_device_name()}, M=5, us per iteration")
    for name, n, k in SHAPES:
        nbytes = n * k * 2
        ncopy = max(4, math.ceil(768e6 / nbytes))
        ws = [ops.preshuffle(torch.randn(n, k, dtype=torch.bfloat16, device="cuda") * 0.02)
              for _ in range(ncopy)]
        wi = [w.view(torch.int32).view(-1) for w in ws]
        x = torch.randn(5, k, dtype=torch.bfloat16, device="cuda")
        waves = ops.decode_waves(name, True, False)
        sink = torch.empty(ncopy, dtype=torch.int64, device="cuda")
        i = [0]

        def gemv():
            j = i[0] = (i[0] + 1) % ncopy
            ops.linear(x, ws[j], waves=waves, preshuffled=True)

        def read_only():
            j = i[0] = (i[0] + 1) % ncopy
            torch.sum(wi[j], dim=0, out=sink[j])

        def warm():
            j = i[0] = (i[0] + 1) % ncopy
            torch.sum(wi[j], dim=0, out=sink[j])
            ops.linear(x, ws[j], waves=waves, preshuffled=True)

        def other():
            j = i[0] = (i[0] + 1) % ncopy
            torch.sum(wi[(j + 1) % ncopy], dim=0, out=sink[j])
            ops.linear(x, ws[j], waves=waves, preshuffled=True)

        t_cold, t_read = timeit(gemv), timeit(read_only)
        t_warm, t_other = timeit(warm), timeit(other)
        print(f"{name:6s} {n:6d}x{k:<6d} {nbytes / 1e6:6.1f} MB | gemv cold {t_cold:6.1f} | "
              f"read {t_read:6.1f} | read+gemv same W {t_warm:6.1f} | read+gemv other W "
              f"{t_other:6.1f} | MALL-warm saves {t_other - t_warm:5.1f} us/call", flush=True)
        del ws, wi


if __name__ == "__main__":
    main()
