"""Decode-GEMV split-K sweep on MI355X (production ops path, pre-shuffled weights).

For every decode projection shape: waves x ksplit grid, M = 1 and 5, cold weights (rotating
copies totalling >= 768 MB, three times the Infinity Cache), median of event-timed loops.
Also checks each split against ksplit = 1 (same inputs) for closeness.

Shapes: Llama-3.1-8B (TP=1), Llama-3-70B per-rank shards at TP=8 and the 70B TP=1 shapes
(``--set 70b``), so the table doubles as the per-rank kernel table of BASELINE configs 4/5.
"""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402

SETS = {
    "8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096),
           ("down", 4096, 14336)],
    "70b-tp8": [("qkv", 1280, 8192), ("o", 8192, 1024), ("gate_up", 7168, 8192),
                ("down", 8192, 3584), ("lm_head", 16032, 8192)],
    "70b": [("qkv", 10240, 8192), ("o", 8192, 8192), ("gate_up", 57344, 8192),
            ("down", 8192, 28672)],
}


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


def sweep(which: str, waves_list=(4, 8, 16), splits=(1, 2, 4), ms=(1, 5)):
    print(f"== split-K GEMV sweep [{which}] (us / weight GB/s); err = max|y - y(ksplit=1)|")
    for name, n, k in SETS[which]:
        nbytes = n * k * 2
        ncopy = max(2, math.ceil(768e6 / nbytes))
        ws = [ops.preshuffle(torch.randn(n, k, dtype=torch.bfloat16, device="cuda") * 0.02)
              for _ in range(ncopy)]
        for m in ms:
            x = torch.randn(m, k, dtype=torch.bfloat16, device="cuda")
            out = torch.empty(m, n, dtype=torch.bfloat16, device="cuda")
            ref = ops.linear(x, ws[0], waves=8, preshuffled=True).float()
            row = f"{name:>8} {n:6d}x{k:<6d} M={m:2d} |"
            for waves in waves_list:
                for ks in splits:
                    i = [0]

                    def f(waves=waves, ks=ks):
                        i[0] = (i[0] + 1) % ncopy
                        ops.linear(x, ws[i[0]], out=out, waves=waves, preshuffled=True, ksplit=ks)
                    try:
                        ops.linear(x, ws[0], out=out, waves=waves, preshuffled=True, ksplit=ks)
                        err = (out.float() - ref).abs().max().item()
                        t = timeit(f)
                        row += f" w{waves}k{ks} {t:6.1f}/{nbytes / t / 1e3:4.0f} e{err:.0e} |"
                    except RuntimeError as e:
                        row += f" w{waves}k{ks} n/a ({str(e)[:20]}) |"
            print(row, flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    assert ops.native_available()
    for which in (sys.argv[1:] or ["8b"]):
        sweep(which)
