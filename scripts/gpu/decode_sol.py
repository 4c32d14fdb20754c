"""Speed-of-light check for the Llama-3.1-8B bf16 decode step on one MI355X.

Replays, in one hipGraph, a chain of plain READ kernels over the exact per-step weight
stream of the fused decode step (per layer: qkv 6144x4096, o 4096x4096, gate_up 28672x4096,
down 4096x14336; then the 128256x4096 LM head) - no math, no attention, no epilogues - and
compares it with one single read of the same 15 GB.  The chain time is what ANY
one-kernel-per-GEMV design pays for the weight stream on this part; the fused decode step
adds attention and epilogues on top (profiles/r2_decode_roofline.md).

Reads are the library's ``stream_read`` probe (16-byte non-temporal loads, 8 in flight per
lane, 2048 workgroups) - the decode GEMVs' load path without their math.  (torch.max over
bf16 only reaches ~2 TB/s and is no ceiling.)
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd import ops  # noqa: E402


def timed(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(iters):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e))
    return statistics.median(res)


def main():
    H, I, V, L = 4096, 14336, 128256, 32
    shapes = []
    for _ in range(L):
        shapes += [(6144, H), (H, H), (2 * I, H), (H, I)]
    shapes.append((V, H))
    bufs = [torch.empty(n * k, dtype=torch.bfloat16, device="cuda").normal_() for n, k in shapes]
    total = sum(b.numel() * 2 for b in bufs)

    nat = ops._native()
    sink = torch.zeros(2048, dtype=torch.int32, device="cuda")

    def chain():  # one read kernel per matrix
        for b in bufs:
            nat.stream_read(b, sink)

    flat = torch.empty(total // 2, dtype=torch.bfloat16, device="cuda").normal_()

    def one_read():
        nat.stream_read(flat, sink)

    t_one = timed(one_read)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        chain()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            chain()
    torch.cuda.current_stream().wait_stream(s)
    t_chain = timed(g.replay)
    print(f"weight stream {total / 1e9:.2f} GB")
    print(f"one read of it:         {t_one:7.3f} ms  ({total / t_one / 1e9:5.2f} TB/s)")
    print(f"{len(bufs)} per-matrix reads (graph): {t_chain:7.3f} ms  "
          f"({total / t_chain / 1e9:5.2f} TB/s)")
    for blocks in (512, 1024, 4096):
        sk = torch.zeros(blocks, dtype=torch.int32, device="cuda")
        t = timed(lambda: nat.stream_read(flat, sk))
        print(f"one read, {blocks:5d} workgroups: {t:7.3f} ms  ({total / t / 1e9:5.2f} TB/s)")


if __name__ == "__main__":
    main()
