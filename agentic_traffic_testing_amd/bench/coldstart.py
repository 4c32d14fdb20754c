"""First-occurrence vs repeat TTFT of the fan-out workload's prefill step shapes.

HIP loads a translation unit's code object at the first launch of one of its kernels
(1.5-2.5 ms each on MI355X), and hipBLASLt loads a solution's code object at its first use,
so any kernel the engine start-up did not touch costs its first timed request that much
(round 5: the first 50- / 95-row burst ran 6.3 / 7.3 ms against 4.7 ms after,
profiles/r5_fanout_ttft_per_episode.txt).  The engine warms every code object it can route
to at start (ops.warm_wide_kernels, decode graph capture); this module proves it: a fresh
engine serves every step shape of bench.py's fan-out episode twice - fresh random tokens each
time, so the prefix cache only hits where the shape says it does - and reports both TTFTs.

Shapes (rows of the prefill step; the kernels they route to at llama-3.1-8b TP=1 bf16):
  planning_17      17 rows, one sequence            fused 16-row-tile GEMVs / wide kernel
  cached_burst     5 x 17 new rows over a cached 560-token prefix   wide kernel (85 rows)
  prefix_560       560 rows, one sequence           mid-M kernel + tuned library GEMMs
  planning_188     188 rows, one sequence           mid-M kernel (o, qkv, down) + library
  burst_475        5 x 95 rows                      mid-M kernel + library
  final_3072       3072 rows, one sequence          tuned library GEMMs + flash prefill

    python -m agentic_traffic_testing_amd.bench.coldstart [--model M] [--reps 2]
"""
from __future__ import annotations

import argparse
import json
import time

import numpy as np

from ..engine.sequence import SamplingParams

SHAPES = ("planning_17", "cached_burst", "prefix_560", "planning_188", "burst_475",
          "final_3072")


def _ttft(eng, prompts, tag: str) -> float:
    """Submit ``prompts`` together (one token each) and return their max TTFT in seconds."""
    t_arr = time.perf_counter()
    rids = [f"{tag}-{i}" for i in range(len(prompts))]
    sp = SamplingParams(temperature=0.2, max_tokens=1, ignore_eos=True, seed=1)
    for rid, p in zip(rids, prompts):
        eng.add_request(rid, p, sp, arrival_time=t_arr)
    done = {}
    while len(done) < len(rids):
        for o in eng.step():
            if o.finished:
                done[o.request_id] = o
    return max(done[r].ttft for r in rids)


def measure(eng, reps: int = 2, seed: int = 0) -> dict:
    """{shape: [TTFT of occurrence 0, 1, ...] in ms} over ``reps`` passes of SHAPES."""
    rng = np.random.default_rng(seed)
    vocab = min(eng.model_cfg.vocab_size, 32000)

    def toks(n):
        return rng.integers(1000, vocab, size=n).tolist()

    out = {s: [] for s in SHAPES}
    for r in range(reps):
        prefix = toks(560)
        out["planning_17"].append(_ttft(eng, [toks(17)], f"p17-{r}"))
        out["prefix_560"].append(_ttft(eng, [prefix], f"pre-{r}"))
        out["cached_burst"].append(_ttft(eng, [prefix + toks(17) for _ in range(5)], f"cb-{r}"))
        out["planning_188"].append(_ttft(eng, [toks(188)], f"p188-{r}"))
        out["burst_475"].append(_ttft(eng, [toks(95) for _ in range(5)], f"b475-{r}"))
        out["final_3072"].append(_ttft(eng, [toks(3072)], f"fin-{r}"))
    return {k: [round(v * 1e3, 3) for v in vs] for k, vs in out.items()}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.1-8B-Instruct")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--max-model-len", type=int, default=4096)
    a = ap.parse_args(argv)
    from ..config import EngineConfig
    from ..engine.llm_engine import LLMEngine

    # bench.py's engine configuration (the headline regime)
    cfg = EngineConfig(model=a.model, dtype="bfloat16", max_model_len=a.max_model_len,
                       max_num_seqs=12, max_num_batched_tokens=8192,
                       gpu_memory_utilization=0.90, use_graphs=True, seed=1234,
                       device="cuda:0")
    t0 = time.perf_counter()
    eng = LLMEngine(cfg)
    eng.runner.capture_all(all_parts=True)
    init_s = time.perf_counter() - t0
    res = measure(eng, a.reps)
    print(json.dumps({"init_s": round(init_s, 2), "ttft_ms": res}), flush=True)


if __name__ == "__main__":
    main()
