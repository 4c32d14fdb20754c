"""Per-workgroup timeline of one wide small-M GEMM launch (ops.set_gemv_trace: [start, K loop
done, split-K partials published, end] on the 100 MHz wall clock per workgroup), cold weights:
where a launch's time goes - dispatch spread, K-loop span, hand-over wait, last-arriver
combine + epilogue.

    python scripts/gpu/wide_timeline.py --proj o --m 85 [--plan 4 4]
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--proj", nargs="+", default=["o", "qkv", "down", "gate_up"])
    ap.add_argument("--m", type=int, nargs="+", default=[85])
    ap.add_argument("--plan", type=int, nargs=2, default=[0, 0])
    a = ap.parse_args()
    assert ops.native_available(), ops._load_error
    ops.ensure_splitk_workspace("cuda")
    dt = torch.bfloat16
    for proj in a.proj:
        n, k = SHAPES[proj]
        ncopy = max(2, int(600e6 // (n * k * 2)) + 1)
        rowmap = "silu" if proj == "gate_up" else "plain"
        wps = [ops.preshuffle((torch.randn(n, k, device="cuda") * 0.02).to(dt), rowmap)
               for _ in range(ncopy)]
        for m in a.m:
            x = torch.randn(m, k, device="cuda").to(dt)
            res = torch.zeros(m, n, dtype=dt, device="cuda")
            act = torch.empty(m, n // 2, dtype=dt, device="cuda")
            tr = torch.zeros(4 * 8192, dtype=torch.int64, device="cuda")

            def run(i, trace=False):
                ops.set_wide_plan(*a.plan)
                if trace:
                    tr.zero_()
                    ops.set_gemv_trace(tr)
                if proj == "gate_up":
                    ops.decode_gate_up_silu(x, wps[i % ncopy], 1e-5, out=act, preshuffled=True)
                else:
                    ops.linear(x, wps[i % ncopy], residual=res, preshuffled=True)
            for i in range(5):
                run(i)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(20):
                run(i)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 20
            run(7, trace=True)
            torch.cuda.synchronize()
            t = tr.view(-1, 4).cpu()
            t = t[t[:, 0] > 0]
            t0 = int(t[:, 0].min())
            st = [(int(r[0]) - t0) / 100 for r in t]
            lp = [(int(r[1]) - int(r[0])) / 100 for r in t]
            pub = [(int(r[2]) - int(r[1])) / 100 for r in t]
            end = [(int(r[3]) - t0) / 100 for r in t]
            last = [(int(r[3]) - int(r[2])) / 100 for r in t if int(r[3]) > int(r[2])]
            print(f"{proj:8s} M={m:4d} plan={a.plan} {us:6.1f} us/call, {len(t)} WGs | start "
                  f"p50/max {q(st, .5):5.2f}/{max(st):5.2f} | K-loop p10/p50/p90 "
                  f"{q(lp, .1):5.2f}/{q(lp, .5):5.2f}/{q(lp, .9):5.2f} | publish p50 "
                  f"{q(pub, .5):5.2f} | last-arriver combine+epilogue p50 "
                  f"{(q(last, .5) if last else 0):5.2f} | end p50/max {q(end, .5):5.2f}/"
                  f"{max(end):5.2f} us", flush=True)
        del wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
