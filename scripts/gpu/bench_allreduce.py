"""Per-call latency / bandwidth of the IPC all-reduce kernels (ops/csrc/allreduce.hip) in the
W-ranks-on-ONE-GPU rehearsal ("no profile records the one-shot kernel's latency
or the two-shot kernel's bandwidth").  Every rank is its own process on cuda:0 (gloo control
group), exactly the TP protocol; the W kernels of one call time-slice ONE device, so these
numbers bound the protocol overhead (flags, uncached peer buffers, rank-ordered fp32 sums),
not xGMI link speed.

Per message size: median us per call of a graph replaying 20 back-to-back calls (graph launch
cost amortised), one-shot for decode messages ([B, 8192] bf16, B = 1..16: the 70B TP=8 X1/X2
shape), two-shot up to prefill messages (1 MiB .. 128 MiB), and the equivalent algorithm
bandwidth 2 (W-1)/W * bytes / t.

    python scripts/gpu/bench_allreduce.py --world 8
"""
import argparse
import os
import socket
import statistics
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


DECODE_ROWS = [1, 2, 5, 8, 16]
PREFILL_MB = [1, 4, 16, 64, 128]


def worker(rank, world, port, q, reps):
    try:
        from agentic_traffic_testing_amd.parallel.comm import init_distributed
        from agentic_traffic_testing_amd.parallel.custom_allreduce import IpcAllReduce

        torch.cuda.set_device(0)
        comm = init_distributed(rank, world, "cuda:0", "gloo", "127.0.0.1", port)
        ar = IpcAllReduce(comm, "cuda:0", max_bytes=16 * 8192 * 2,
                          large_max_bytes=max(PREFILL_MB) << 20)
        out = []
        cases = [("oneshot", r * 8192, f"[{r}, 8192]") for r in DECODE_ROWS]
        cases += [("twoshot", r * 8192, f"[{r}, 8192]") for r in DECODE_ROWS]
        cases += [("twoshot", (mb << 20) // 2, f"{mb} MiB") for mb in PREFILL_MB]
        s = torch.cuda.Stream()
        for mode, n, label in cases:
            x = torch.ones(n, dtype=torch.bfloat16, device="cuda")
            calls = 20
            with torch.cuda.stream(s):
                ar.all_reduce(x, mode)  # warm
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(calls):
                    ar.all_reduce(x, mode)
            ts = []
            for _ in range(reps):
                comm.barrier()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / calls)
            out.append((mode, label, n * 2, statistics.median(ts)))
            del g
        err = ar.check()
        comm.barrier()
        ar.close()
        q.put((rank, out, err))
        torch.distributed.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), -1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    print("# IPC all-reduce, W ranks on ONE MI355X (time-sliced: protocol cost, not xGMI); "
          "us per call = graph of 20 back-to-back calls / 20, median of reps; algbw = "
          "2(W-1)/W * bytes / t")
    for world in a.world:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = free_port()
        ps = [ctx.Process(target=worker, args=(r, world, port, q, a.reps)) for r in range(world)]
        for p in ps:
            p.start()
        res = sorted(q.get(timeout=600) for _ in ps)
        for p in ps:
            p.join(timeout=60)
        for rank, out, err in res:
            if err == -1 or isinstance(out, str):
                raise SystemExit(f"rank {rank} failed: {out}")
        # per case: the slowest rank's time (the collective completes when every rank did)
        for i, (mode, label, nbytes, _) in enumerate(res[0][1]):
            t = max(r[1][i][3] for r in res)
            bw = 2 * (world - 1) / world * nbytes / (t * 1e-6) / 1e9
            print(f"W={world} {mode:8s} {label:>12s} {nbytes / 1024:10.0f} KiB | {t:9.2f} us/call | "
                  f"algbw {bw:8.1f} GB/s", flush=True)
        assert all(r[2] == 0 for r in res), "a bounded wait timed out"


if __name__ == "__main__":
    main()
