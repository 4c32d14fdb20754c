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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    ba = bench.parse_args([])
    eng = LLMEngine(bench._cfg(ba, "cuda"))
    wl = FanoutWorkload(eng, fanout=ba.fanout, max_tokens=ba.max_tokens, seed=0)
    for _ in range(a.warmup):
        wl.run_episode()
    for e in range(a.episodes):
        r = wl.run_episode()
        for name, rows, cached, ttfts in r.phases:
            print(f"episode {e} {name:8s} prompt {rows:5d} cached {cached:5d} ttft ms "
                  + " ".join(f"{1e3 * t:6.2f}" for t in ttfts), flush=True)


if __name__ == "__main__":
    main()
