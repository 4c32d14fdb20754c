"""TunableOp (rocBLAS + hipBLASLt solution search) vs the default hipBLASLt heuristic on the
Llama-3.1-8B prefill projections at the fan-out workload's row counts (planning ~73, burst
~382, final ~3092).  Cold weights (rotating copies past the Infinity Cache).  Writes the tuned
table to $TUNABLEOP_CSV (default gpurun_out/tunableop_8b.csv).

    python scripts/gpu/probe_tunableop.py --m 73 382 1000 3092
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timed(fn, iters=20):
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
    ap.add_argument("--m", type=int, nargs="+", default=[73, 382, 1000, 3092])
    a = ap.parse_args()
    tun = torch.cuda.tunable
    csv = os.environ.get("TUNABLEOP_CSV", "gpurun_out/tunableop_8b.csv")
    res = {}
    data = {}
    for name, (n, k) in SHAPES.items():
        copies = max(2, int(768e6 / (n * k * 2)) + 1)
        ws = [(torch.rand(n, k, device="cuda") * 2 - 1).to(torch.bfloat16) / k ** 0.5
              for _ in range(copies)]
        for m in a.m:
            x = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
            data[(name, m)] = (x, ws)
    for tuned in (False, True):
        tun.enable(tuned)
        tun.tuning_enable(tuned)
        if tuned:
            tun.set_filename(csv)
            tun.set_max_tuning_duration(60)
        for (name, m), (x, ws) in data.items():
            fn = lambda i, x=x, ws=ws: torch.nn.functional.linear(x, ws[i % len(ws)])  # noqa
            if tuned:
                for w in ws[:1]:
                    torch.nn.functional.linear(x, w)  # the tuning call
            res[(name, m, tuned)] = timed(fn)
    for (name, m), _ in data.items():
        n, k = SHAPES[name]
        d, t = res[(name, m, False)], res[(name, m, True)]
        tf = 2 * m * n * k / t / 1e6
        print(f"{name:8s} M={m:5d} N={n:6d} K={k:6d} | hipBLASLt default {d:8.1f} us | "
              f"TunableOp {t:8.1f} us ({tf:5.0f} TF) | {d / t:5.2f}x", flush=True)
    # the tuned table (solution names per shape) goes to `csv` when the process exits


if __name__ == "__main__":
    main()
