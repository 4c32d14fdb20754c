"""Bandwidth of the prefill elementwise kernels at the fan-out workload's row counts:
silu_and_mul ([M, 2 I] -> [M, I]) and the fused residual-add RMSNorm ([M, H]).  Reports us per
call and the achieved HBM rate (bytes read + written / t) against ~6 TB/s.

    python scripts/gpu/probe_elementwise.py --m 382 3200
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402


def timed(fn, iters=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[382, 3200])
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--hidden", type=int, default=4096)
    a = ap.parse_args()
    for m in a.m:
        # several copies so consecutive calls do not hit the Infinity Cache
        copies = max(2, int(600e6 / (m * 2 * a.inter * 2)) + 1)
        xs = [torch.randn(m, 2 * a.inter, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
        outs = [torch.empty(m, a.inter, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
        i = [0]

        def silu():
            k = i[0] % copies
            i[0] += 1
            ops.silu_and_mul(xs[k], out=outs[k])

        ref = torch.nn.functional.silu(xs[0][:, :a.inter].float()) * xs[0][:, a.inter:].float()
        ops.silu_and_mul(xs[0], out=outs[0])
        err = ((outs[0].float() - ref).abs().max() / ref.abs().max()).item()
        t = timed(silu)
        nbytes = m * a.inter * 2 * 3
        print(f"silu_and_mul M={m:5d} I={a.inter} | {t:8.1f} us | {nbytes / t / 1e6:6.2f} TB/s | "
              f"rel err {err:.1e}", flush=True)
        del xs, outs
        copies = max(2, int(600e6 / (m * a.hidden * 2 * 3)) + 1)
        hs = [torch.randn(m, a.hidden, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
        rs = [torch.randn(m, a.hidden, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
        w = torch.randn(a.hidden, device="cuda", dtype=torch.bfloat16)

        def norm():
            k = i[0] % copies
            i[0] += 1
            ops.fused_add_rms_norm(hs[k], rs[k], w, 1e-5)

        t = timed(norm)
        nbytes = m * a.hidden * 2 * 4  # x, residual in; residual, out written
        print(f"add_rms_norm M={m:5d} H={a.hidden} | {t:8.1f} us | {nbytes / t / 1e6:6.2f} TB/s",
              flush=True)
        del hs, rs


if __name__ == "__main__":
    main()
