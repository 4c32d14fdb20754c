"""Why a 17-row step of the fused decode GEMVs costs ~1.8x a 16-row one (gate_up 69 vs 39 us):
times ops.decode_gate_up_silu on the pre-shuffled 8B gate_up at M = 8, 16, 17, 24, 32 (cold
weights: rotating copies), for a PMC pass with --only-m.

    python scripts/gpu/probe_skinny_mt.py [--only-m 17]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402


def sweep_linear():
    """waves sweep for the residual-epilogue projections (o, down; qkv as a plain GEMV) at
    1-2 MFMA row blocks, pre-shuffled bf16 8B shapes, cold weights."""
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336)}
    for proj, (n, k) in shapes.items():
        ws = [ops.preshuffle((torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16))
              for _ in range(4)]
        for m in (16, 17, 32):
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            res = torch.zeros(m, n, device="cuda", dtype=torch.bfloat16)
            row = []
            for waves in (4, 8, 16):
                def run(i):
                    ops.linear(x, ws[i % 4], residual=res, waves=waves, preshuffled=True,
                               ksplit=None, proj=proj)
                for i in range(3):
                    run(i)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(40):
                    run(i)
                e1.record()
                torch.cuda.synchronize()
                row.append(f"w{waves}={e0.elapsed_time(e1) * 1e3 / 40:6.1f}us")
            print(f"{proj:5s} M={m:3d}: " + "  ".join(row), flush=True)


def time_qkv_rope():
    """fused RMSNorm + QKV + RoPE + KV write (8B shapes, pre-shuffled) at 16 / 17 / 32 rows;
    the wave count comes from ops.decode_waves (ATTA_DECODE_WAVES=qkv.ps=N to sweep)."""
    n, k, hq, hkv, bs, nb = 6144, 4096, 32, 8, 16, 64
    ws = [ops.preshuffle((torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16), "qkv")
          for _ in range(4)]
    kc = torch.zeros(nb, hkv, bs, 128, dtype=torch.bfloat16, device="cuda")
    vc = torch.zeros(nb, hkv, 128, bs, dtype=torch.bfloat16, device="cuda")
    cs = ops.ref.rope_cos_sin(128, 4096, 500000.0, None, device="cuda")
    for m in (16, 17, 32):
        x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
        pos = torch.arange(m, dtype=torch.int32, device="cuda")
        slots = torch.arange(m, dtype=torch.int32, device="cuda")
        q = torch.empty(m, hq, 128, dtype=torch.bfloat16, device="cuda")

        def run(i):
            ops.decode_qkv_rope(x, ws[i % 4], 1e-5, pos, slots, cs, kc, vc, hq, hkv, q_out=q,
                                preshuffled=True)
        for i in range(3):
            run(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(40):
            run(i)
        e1.record()
        torch.cuda.synchronize()
        print(f"qkv_rope waves={ops.decode_waves('qkv', True)} M={m:3d}: "
              f"{e0.elapsed_time(e1) * 1e3 / 40:6.1f} us", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only-m", type=int, default=0)
    ap.add_argument("--sweep-linear", action="store_true")
    ap.add_argument("--qkv-rope", action="store_true")
    a = ap.parse_args()
    if a.sweep_linear:
        sweep_linear()
        return
    if a.qkv_rope:
        time_qkv_rope()
        return
    n, k = 28672, 4096
    copies = 4
    ws = [ops.preshuffle((torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16), "silu")
          for _ in range(copies)]
    for m in ([a.only_m] if a.only_m else [8, 16, 17, 24, 32]):
        x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
        out = torch.empty(m, n // 2, device="cuda", dtype=torch.bfloat16)
        for i in range(3):
            ops.decode_gate_up_silu(x, ws[i % copies], 1e-5, out=out, preshuffled=True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        iters = 40
        for i in range(iters):
            ops.decode_gate_up_silu(x, ws[i % copies], 1e-5, out=out, preshuffled=True)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e3 / iters
        print(f"gate_up+silu M={m:3d}: {t:7.1f} us ({n * k * 2 / t / 1e6:5.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
