"""Prefill attention microbench on MI355X: flash (LDS-staged, 32x32x16 MFMA) vs v1, causal,
one sequence of N tokens (plus a chunk-after-prefix case), Llama-3-8B (32/8) and 70B (64/8)
head geometry.  Reports us and TFLOP/s (causal FLOPs = 2 * 2 * N^2/2 * D * Hq)."""
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from agentic_traffic_testing_amd import ops  # noqa: E402
from test_kernels_gpu import _make_paged, _tiles  # noqa: E402


GRAPH = False


def timeit(fn, iters=20, reps=3):
    """us per call; with --graph the iters calls replay from one hipGraph (GPU time without
    the host launch cost, which dominates the small burst shapes in eager mode)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = None
    if GRAPH:
        g = torch.cuda.CUDAGraph()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
            for _ in range(iters):
                fn()
        torch.cuda.current_stream().wait_stream(st)
        g.replay()
        torch.cuda.synchronize()
    res = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        if g is not None:
            g.replay()
        else:
            for _ in range(iters):
                fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / iters * 1000)
    return statistics.median(res)


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--impls", nargs="+", default=["flash", "v1"])
    ap.add_argument("--hq", type=int, nargs="+", default=[32, 64])
    ap.add_argument("--n", type=int, nargs="+", default=[0],
                    help="causal sequence lengths (0 = the default shape list)")
    ap.add_argument("--multi", nargs="+", default=[],
                    help="batched steps KV:Q:N - N sequences of Q new tokens over KV keys each "
                         "(the cached burst: 617:17:5)")
    ap.add_argument("--graph", action="store_true", help="time hipGraph replays")
    a = ap.parse_args()
    global GRAPH
    GRAPH = a.graph
    shapes = ((512, 512), (2600, 2600), (4096, 4096), (3000 + 700, 700), (8192, 8192))
    if a.n != [0]:
        shapes = tuple((n, n) for n in a.n)
    steps = [[s] for s in shapes]
    for m in a.multi:
        kv_, q_, n_ = (int(v) for v in m.split(":"))
        steps.append([(kv_, q_)] * n_)
    if a.multi and a.n == [0]:
        steps = steps[len(shapes):]
    dt = torch.bfloat16
    print("== prefill attention (us / TFLOP/s)")
    for hq, hkv in ((h, 8) for h in a.hq):
        for seqs in steps:
            k, v, bt, kvlen, qstart, T = _make_paged(seqs, hkv, 16, dt)
            q = torch.randn(T, hq, 128, dtype=dt, device="cuda")
            flops = sum(4 * 128 * hq * (ql * (kv - ql) + ql * (ql + 1) / 2) for kv, ql in seqs)
            kv, ql = seqs[0]
            row = f"Hq={hq:2d} kv={kv:5d} q={ql:5d} x{len(seqs)} |"
            for impl in a.impls:
                ts, to = _tiles(seqs, ops.prefill_tile_tokens(hq // hkv, impl))
                out = torch.empty_like(q)
                t = timeit(lambda: ops.attention_prefill(q, k, v, bt, kvlen, qstart, ts, to,
                                                         0.088, out=out, impl=impl))
                row += f" {impl} {t:8.1f} us {flops / t / 1e6:6.1f} TF |"
            print(row, flush=True)


if __name__ == "__main__":
    assert ops.native_available()
    main()
