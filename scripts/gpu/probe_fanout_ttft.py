"""Per-episode TTFT of the fan-out workload (bench.py's engine regime): every request's TTFT
by phase for each timed episode, so a p50 shift can be traced to the episodes / phases that
moved.

    python scripts/gpu/probe_fanout_ttft.py --episodes 3 --warmup 5
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import bench  # noqa: E402  (the headline's engine config)
from agentic_traffic_testing_amd.bench.fanout import FanoutWorkload  # noqa: E402
from agentic_traffic_testing_amd.engine.llm_engine import LLMEngine  # noqa: E402


STEPS = []


def _instrument(eng):
    """Time the host and GPU parts of every prefill step (ms): step entry -> forward launch
    start (schedule + metadata), the forward's launch loop, GPU time of the forward (events),
    and launch end -> tokens on the host."""
    import time
    import torch
    r = eng.runner
    orig_run, orig_exec = r._run, r.execute
    cur = {}

    def run(hdr):
        cur["t_run"] = time.perf_counter()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig_run(hdr)
        e1.record()
        cur["t_launched"] = time.perf_counter()
        cur["ev"] = (e0, e1)
        return out

    def execute(batch):
        t0 = time.perf_counter()
        out = orig_exec(batch)
        t1 = time.perf_counter()
        if batch.num_decode < len(batch.seqs) and "t_run" in cur:
            e0, e1 = cur["ev"]
            STEPS.append({"rows": float(sum(batch.q_len)),
                          "host_pre": 1e3 * (cur["t_run"] - t0),
                          "launch_loop": 1e3 * (cur["t_launched"] - cur["t_run"]),
                          "gpu_fwd": e0.elapsed_time(e1),
                          "execute": 1e3 * (t1 - t0)})
        cur.clear()
        return out

    r._run, r.execute = run, execute


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--host", action="store_true", help="time host / GPU parts of prefill steps")
    a = ap.parse_args()
    ba = bench.parse_args([])
    eng = LLMEngine(bench._cfg(ba, "cuda"))
    wl = FanoutWorkload(eng, fanout=ba.fanout, max_tokens=ba.max_tokens, seed=0)
    for _ in range(a.warmup):
        wl.run_episode()
    if a.host:
        _instrument(eng)
    for e in range(a.episodes):
        r = wl.run_episode()
        for name, rows, cached, ttfts in r.phases:
            print(f"episode {e} {name:8s} prompt {rows:5d} cached {cached:5d} ttft ms "
                  + " ".join(f"{1e3 * t:6.2f}" for t in ttfts), flush=True)
        for rec in STEPS:
            print("  prefill step: " + ", ".join(f"{k} {v:.3f}" for k, v in rec.items()),
                  flush=True)
        STEPS.clear()


if __name__ == "__main__":
    main()
