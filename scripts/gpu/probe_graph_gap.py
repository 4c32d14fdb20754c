#!/usr/bin/env python3
"""Replay-to-replay cost of hipGraphs on this stack: how long does the GPU sit between the last
kernel of one graph replay and the first kernel of the next when the host has queued both long
before?  (The headline bench idles ~19-36 us per decode step at that boundary,
profiles/r5_decode_idle_gaps.txt.)

Cases, each timed with events around R back-to-back replays (host far ahead of the GPU):
  one graph of N kernels, replayed R times               -> (t - R * N * k) / R per boundary
  two graphs alternated                                   -> same, different exec each time
  stream copies (pinned H2D + D2H) around every replay    -> the shipped decode step's shape
  one graph holding 4 consecutive "steps" (4 N kernels)   -> R / 4 boundaries
  copies + event records as ModelRunner.launch() issues them

    python scripts/gpu/probe_graph_gap.py
"""
import torch


def main():
    dev = torch.device("cuda")
    x = torch.zeros(1 << 16, device=dev)
    host = torch.zeros(4096, dtype=torch.int32, pin_memory=True)
    dmeta = torch.zeros(4096, dtype=torch.int32, device=dev)
    toks = torch.zeros(256, dtype=torch.int64, device=dev)
    htoks = torch.zeros(256, dtype=torch.int64, pin_memory=True)
    N, R = 160, 200  # ~ a decode step's kernel count (5 per layer x 32)

    def step():
        for _ in range(N):
            x.add_(1.0)

    def capture(fn):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        torch.cuda.synchronize()
        return g

    def timed(body, reps):
        body()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(reps):
            body(i)
        b.record()
        b.synchronize()
        return a.elapsed_time(b) * 1e3  # us

    # per-kernel time inside a graph: one graph of 4 N kernels, few replays
    g4 = capture(lambda: [step() for _ in range(4)])
    t4 = timed(lambda i=0: g4.replay(), R // 4)
    per_kernel = t4 / (R // 4) / (4 * N)
    g1 = capture(step)
    g2 = capture(step)
    t1 = timed(lambda i=0: g1.replay(), R)
    t2 = timed(lambda i=0: (g1 if i % 2 == 0 else g2).replay(), R)

    def with_copies(i=0):
        dmeta.copy_(host, non_blocking=True)
        g1.replay()
        htoks.copy_(toks, non_blocking=True)

    t3 = timed(with_copies, R)
    evs = [torch.cuda.Event() for _ in range(4)]

    def copies_two_events(i=0):  # the shipped launch(): H2D, event, replay, D2H, event
        dmeta.copy_(host, non_blocking=True)
        evs[(i % 2) * 2].record()
        g1.replay()
        htoks.copy_(toks, non_blocking=True)
        evs[(i % 2) * 2 + 1].record()

    def copies_one_event(i=0):  # the token event alone also orders the metadata buffer reuse
        dmeta.copy_(host, non_blocking=True)
        g1.replay()
        htoks.copy_(toks, non_blocking=True)
        evs[(i % 2) * 2 + 1].record()

    t5 = timed(copies_two_events, R)
    t6 = timed(copies_one_event, R)
    base = N * per_kernel
    print(f"kernel in graph: {per_kernel:.2f} us each ({N} per step)")
    print(f"one graph replayed        : {t1 / R:8.1f} us per step -> boundary {t1 / R - base:6.1f} us")
    print(f"two graphs alternated     : {t2 / R:8.1f} us per step -> boundary {t2 / R - base:6.1f} us")
    print(f"stream copies around each : {t3 / R:8.1f} us per step -> boundary {t3 / R - base:6.1f} us")
    print(f"4 steps in one graph      : {t4 / R:8.1f} us per step -> boundary "
          f"{t4 / R - base:6.1f} us")
    print(f"copies + 2 event records  : {t5 / R:8.1f} us per step -> boundary {t5 / R - base:6.1f} us")
    print(f"copies + 1 event record   : {t6 / R:8.1f} us per step -> boundary {t6 / R - base:6.1f} us")


if __name__ == "__main__":
    main()
