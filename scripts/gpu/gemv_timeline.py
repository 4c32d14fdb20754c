#!/usr/bin/env python3
"""Per-workgroup timeline of a chain of decode GEMV launches replayed from one hipGraph
(ops.set_gemv_trace): where the ~4 us per launch above a single monolithic weight read go
(profiles/r2_decode_roofline.md).  Llama-3.1-8B decode shapes at B rows (pre-shuffled bf16
weights, L distinct layers so nothing is cache-resident): per layer qkv+RoPE (4 waves), o+res
(8), gate_up+SiLU (16), down+res (8); attention is left out so every boundary is GEMV ->
GEMV.

Per launch (wall clock, 100 MHz = 10 ns): workgroups, dispatch spread (last - first start),
median workgroup span, drain (last end - median end), launch gap (this launch's first start -
the previous launch's last end), and the launch's HBM rate over its first-start -> last-end
window.
"""
import argparse
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402

H, I, NQ, NKV, BS = 4096, 14336, 32, 8, 16


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1)
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--replays", type=int, default=20)
    a = ap.parse_args()
    dev, dt = "cuda", torch.bfloat16
    B = a.rows
    torch.manual_seed(0)
    layers = []
    for _ in range(a.layers):
        layers.append(dict(
            qkv=ops.preshuffle((torch.randn((NQ + 2 * NKV) * 128, H, device=dev) / 64).to(dt), "qkv"),
            o=ops.preshuffle((torch.randn(H, NQ * 128, device=dev) / 64).to(dt)),
            gu=ops.preshuffle((torch.randn(2 * I, H, device=dev) / 64).to(dt), "silu"),
            down=ops.preshuffle((torch.randn(H, I, device=dev) / 64).to(dt))))
    x = torch.randn(B, H, device=dev).to(dt)
    q = torch.empty(B, NQ, 128, device=dev, dtype=dt)
    act = torch.empty(B, I, device=dev, dtype=dt)
    kc = torch.zeros(64, NKV, BS, 128, device=dev, dtype=dt)
    vc = torch.zeros(64, NKV, 128, BS, device=dev, dtype=dt)
    pos = torch.full((B,), 7, dtype=torch.int32, device=dev)
    slots = torch.arange(B, dtype=torch.int32, device=dev)
    cs = torch.randn(4096, 128, device=dev)
    launches = []  # (name, grid, bytes, trace)
    for li in range(a.layers):
        for name, rows, k in (("qkv", (NQ + 2 * NKV) * 128, H), ("o", H, NQ * 128),
                              ("gate_up", 2 * I, H), ("down", H, I)):
            grid = rows // 16
            launches.append((name, grid, rows * k * 2,
                             torch.zeros(grid, 2, dtype=torch.int64, device=dev)))

    def chain(trace=True):
        it = iter(launches)

        def tr():
            t = next(it)[3]
            ops.set_gemv_trace(t if trace else None)

        for L in layers:
            tr()
            ops.decode_qkv_rope(x, L["qkv"], 1e-5, pos, slots, cs, kc, vc, NQ, NKV, q_out=q,
                                preshuffled=True)
            tr()
            ops.linear(q.view(B, NQ * 128), L["o"], residual=x, waves=ops.decode_waves("o", True),
                       preshuffled=True, ksplit=None, proj="o")
            tr()
            ops.decode_gate_up_silu(x, L["gu"], 1e-5, out=act, preshuffled=True)
            tr()
            ops.linear(act, L["down"], residual=x, waves=ops.decode_waves("down", True),
                       preshuffled=True, ksplit=None, proj="down")

    chain()  # warm-up (eager), then capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            chain()
    g0 = torch.cuda.CUDAGraph()  # the same chain without the probe
    with torch.cuda.stream(s):
        with torch.cuda.graph(g0, stream=s):
            chain(trace=False)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def timed(graph):
        out = []
        for _ in range(a.replays):
            e0.record()
            graph.replay()
            e1.record()
            torch.cuda.synchronize()
            out.append(e0.elapsed_time(e1) * 1e3)
        return statistics.median(out)

    plain = timed(g0)
    spans = [timed(g)]
    total_bytes = sum(b for _, _, b, _ in launches)
    print(f"# decode GEMV chain, B={B}, {a.layers} layers x 4 launches, one hipGraph; replay "
          f"median {statistics.median(spans):.1f} us for {total_bytes / 1e6:.0f} MB "
          f"({total_bytes / statistics.median(spans) / 1e6:.2f} TB/s; without the probe "
          f"{plain:.1f} us, {total_bytes / plain / 1e6:.2f} TB/s); last replay's timeline:")
    print(f"{'launch':10s} {'WGs':>5s} {'gap':>6s} {'spread':>7s} {'wg_med':>7s} {'drain':>6s} "
          f"{'window':>7s} {'TB/s':>5s}   (us)")
    prev_end = None
    first = None
    rows = []
    for name, grid, nbytes, tr in launches:
        t = tr.cpu().double() / 100.0  # us
        st, en = t[:, 0], t[:, 1]
        if first is None:
            first = float(st.min())
        med_end = float(en.median())
        gap = float(st.min()) - prev_end if prev_end is not None else float("nan")
        window = float(en.max() - st.min())
        if window <= 0:  # launch without the probe (e.g. the persistent gate_up variant)
            print(f"{name:10s} {grid:5d}   (no timeline)")
            prev_end = None
            rows.append((float("nan"), 0.0, 0.0, 0.0, 0.0))
            continue
        rows.append((gap, float(st.max() - st.min()), float((en - st).median()),
                     float(en.max()) - med_end, window))
        print(f"{name:10s} {grid:5d} {gap:6.2f} {rows[-1][1]:7.2f} {rows[-1][2]:7.2f} "
              f"{rows[-1][3]:6.2f} {window:7.2f} {nbytes / window / 1e6:5.2f}")
        prev_end = float(en.max())
    gaps = [r[0] for r in rows[1:] if r[0] == r[0]] or [0.0]
    print(f"# chain span {prev_end - first:.1f} us; launch gaps sum {sum(gaps):.1f} us "
          f"(median {statistics.median(gaps):.2f}); dispatch spreads sum "
          f"{sum(r[1] for r in rows):.1f}; drains sum {sum(r[3] for r in rows):.1f}")
    ops.set_gemv_trace(None)


if __name__ == "__main__":
    main()
