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
    python scripts/gpu/bench_allreduce.py --world 2 4 8 --distinct   # 8-GPU node: rank r on
        cuda:r over xGMI, RCCL (nccl) control group, and RCCL all_reduce timed beside the IPC
        kernels (scripts/gpu/scale.sh)
"""
import argparse
import json
import os
import socket
import statistics
import sys
import time

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


DECODE_ROWS = [1, 2, 5, 8, 16]
PREFILL_MB = [1, 4, 16, 64, 128]


def worker(rank, world, port, q, reps, distinct=False):
    try:
        import torch.distributed as dist

        from agentic_traffic_testing_amd.parallel.comm import init_distributed
        from agentic_traffic_testing_amd.parallel.custom_allreduce import IpcAllReduce

        dev = f"cuda:{rank}" if distinct else "cuda:0"
        torch.cuda.set_device(dev)
        comm = init_distributed(rank, world, dev, "nccl" if distinct else "gloo", "127.0.0.1",
                                port)
        ar = IpcAllReduce(comm, dev, max_bytes=16 * 8192 * 2,
                          large_max_bytes=max(PREFILL_MB) << 20)
        out = []
        cases = [("oneshot", r * 8192, f"[{r}, 8192]") for r in DECODE_ROWS]
        cases += [("twoshot", r * 8192, f"[{r}, 8192]") for r in DECODE_ROWS]
        cases += [("twoshot", (mb << 20) // 2, f"{mb} MiB") for mb in PREFILL_MB]
        if distinct:  # RCCL ring / tree over xGMI, same messages
            cases += [("rccl", r * 8192, f"[{r}, 8192]") for r in DECODE_ROWS]
            cases += [("rccl", (mb << 20) // 2, f"{mb} MiB") for mb in PREFILL_MB]

        def call(x, mode):
            if mode == "rccl":
                dist.all_reduce(x)
            else:
                ar.all_reduce(x, mode)

        s = torch.cuda.Stream()
        for mode, n, label in cases:
            x = torch.ones(n, dtype=torch.bfloat16, device="cuda")
            calls = 20
            with torch.cuda.stream(s):
                call(x, mode)  # warm
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(calls):
                    call(x, mode)
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


def cpu_twin_worker(rank, world, port, q, reps):
    """--cpu-twin: the same cases through gloo all_reduce on CPU tensors (protocol rehearsal
    of the JSON contract for tests/test_scale_recipe.py; says nothing about GPU speed)."""
    try:
        import torch.distributed as dist

        from agentic_traffic_testing_amd.parallel.comm import init_distributed

        comm = init_distributed(rank, world, "cpu", "gloo", "127.0.0.1", port)
        out = []
        for r in DECODE_ROWS[:2]:
            x = torch.ones(r * 8192, dtype=torch.float32)
            ts = []
            for _ in range(reps):
                comm.barrier()
                t0 = time.perf_counter()
                dist.all_reduce(x)
                ts.append((time.perf_counter() - t0) * 1e6)
            out.append(("gloo", f"[{r}, 8192]", x.numel() * 2, statistics.median(ts)))
        comm.barrier()
        q.put((rank, out, 0))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, repr(e) + traceback.format_exc(), -1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--distinct", action="store_true",
                    help="rank r on cuda:r (needs W GPUs): the IPC kernels over xGMI + RCCL")
    ap.add_argument("--json", action="store_true", help="one JSON line per case")
    ap.add_argument("--cpu-twin", action="store_true",
                    help="gloo on CPU tensors: the JSON contract without a GPU")
    a = ap.parse_args()
    if a.json:
        pass
    elif a.distinct:
        print("# IPC all-reduce vs RCCL, rank r on cuda:r (xGMI); us per call = graph of 20 "
              "back-to-back calls / 20, median of reps; algbw = 2(W-1)/W * bytes / t")
    else:
        print("# IPC all-reduce, W ranks on ONE MI355X (time-sliced: protocol cost, not xGMI); "
              "us per call = graph of 20 back-to-back calls / 20, median of reps; algbw = "
              "2(W-1)/W * bytes / t")
    have = 64 if a.cpu_twin else torch.cuda.device_count()
    for world in a.world:
        if a.distinct and world > have:
            print(json.dumps({"world": world, "skipped": f"{have} GPU(s) visible"}) if a.json
                  else f"W={world} skipped: {have} GPU(s) visible", flush=True)
            continue
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = free_port()
        ps = [(ctx.Process(target=cpu_twin_worker, args=(r, world, port, q, a.reps))
              if a.cpu_twin else
              ctx.Process(target=worker, args=(r, world, port, q, a.reps, a.distinct))) for r in range(world)]
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
            if a.json:
                print(json.dumps({"world": world, "mode": mode, "message": label,
                                  "bytes": nbytes, "us_per_call": round(t, 2),
                                  "algbw_GBps": round(bw, 1),
                                  "devices": "distinct" if a.distinct else
                                  ("cpu" if a.cpu_twin else "one GPU")}), flush=True)
                continue
            print(f"W={world} {mode:8s} {label:>12s} {nbytes / 1024:10.0f} KiB | {t:9.2f} us/call | "
                  f"algbw {bw:8.1f} GB/s", flush=True)
        assert all(r[2] == 0 for r in res), "a bounded wait timed out"


if __name__ == "__main__":
    main()
