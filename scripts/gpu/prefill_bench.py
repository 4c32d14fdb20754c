"""Prefill (TTFT) microbenchmark on MI355X: one fresh prompt of N tokens through the engine,
max_tokens 1, prefix cache off so every run computes the whole prompt.

Prints median wall ms per prefill for each N; run under ``rocprofv3 --kernel-trace --stats``
for the per-kernel split (scripts/gpu/profile_prefill.sh)."""
import argparse
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from agentic_traffic_testing_amd.config import EngineConfig  # noqa: E402
from agentic_traffic_testing_amd.engine.llm_engine import LLMEngine  # noqa: E402
from agentic_traffic_testing_amd.engine.sequence import SamplingParams  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3.1-8b")
    ap.add_argument("--tokens", default="512,2600")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--quantization", default="")
    ap.add_argument("--set", action="append", default=[],
                    help="EngineConfig override key=value (ints / floats / strings)")
    ap.add_argument("--seqs", type=int, default=1,
                    help="split each N into this many prompts prefilled together (5 = the "
                         "fan-out burst shape)")
    a = ap.parse_args()
    cfg = EngineConfig(model=a.model, max_model_len=8192, max_num_batched_tokens=8192,
                       enable_prefix_caching=False, quantization=a.quantization,
                       num_kv_blocks=4096)
    for kv in a.set:
        k, v = kv.split("=", 1)
        cur = getattr(cfg, k)
        setattr(cfg, k, type(cur)(v) if not isinstance(cur, bool) else v in ("1", "true"))
    eng = LLMEngine(cfg)
    rng = np.random.default_rng(0)
    sp = SamplingParams(temperature=0.2, max_tokens=1, ignore_eos=True)
    # window markers for rocprof summaries (scripts/gpu/summarize_trace.py --window): one
    # stream_read_kernel dispatch brackets each measured (post-warm-up) region, so model init,
    # random-weight generation and the warm-up prefill never enter a profile table
    buf = torch.zeros(4096, dtype=torch.int32, device="cuda")
    sink = torch.zeros(1, dtype=torch.int32, device="cuda")

    def marker():
        torch.ops.atta.stream_read(buf, sink)
        torch.cuda.synchronize()

    for n in map(int, a.tokens.split(",")):
        times = []
        for r in range(a.reps + 1):
            prompts = [rng.integers(1000, 100000, size=n // a.seqs).tolist()
                       for _ in range(a.seqs)]
            torch.cuda.synchronize()
            if r == 1:
                marker()
            t0 = time.perf_counter()
            eng.generate(prompts, sp)
            torch.cuda.synchronize()
            if r:
                times.append((time.perf_counter() - t0) * 1e3)
        marker()
        print(f"prefill {n:6d} tokens ({a.seqs} seqs): {statistics.median(times):8.2f} ms "
              f"({n / statistics.median(times) * 1e3:9.0f} tok/s)", flush=True)


if __name__ == "__main__":
    main()
