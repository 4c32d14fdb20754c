#!/usr/bin/env python3
"""Phase timeline of the persistent decode step (ops/csrc/decode_step.hip) on the headline
model: per phase kind the critical-path time (latest workgroup end of the phase minus the
latest end of the phase before it), against the weight-streaming time of its bytes at the
box's read rate, plus where the loader / compute waves waited.

    python scripts/gpu/mk_profile.py [--model llama-3.1-8b] [--ctx 3000] [--rows 1 5]
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from agentic_traffic_testing_amd import ops  # noqa: E402
from agentic_traffic_testing_amd.config import EngineConfig  # noqa: E402
from agentic_traffic_testing_amd.engine.llm_engine import LLMEngine  # noqa: E402
from agentic_traffic_testing_amd.engine.sequence import SamplingParams  # noqa: E402

KINDS = ["QKV", "ATT", "O", "GU", "DOWN"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.1-8B-Instruct")
    ap.add_argument("--ctx", type=int, default=3000)
    ap.add_argument("--rows", type=int, nargs="+", default=[1, 5])
    ap.add_argument("--steps", type=int, default=48)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    G = ops.decode_step_grid()
    from agentic_traffic_testing_amd.config import resolve_model
    mc, _ = resolve_model(a.model)
    L = mc.num_layers
    NP = 3 + 5 * L
    trace = torch.zeros(G, NP, 2, dtype=torch.int64, device="cuda")
    stats = torch.zeros(G, 4, dtype=torch.int64, device="cuda")
    ops.set_decode_step_trace(trace, stats)
    eng = LLMEngine(EngineConfig(model=a.model, device="cuda", max_model_len=4096,
                                 max_num_seqs=12, decode_megakernel=True))
    r = eng.runner
    assert r.mk_sync is not None, "megakernel not enabled"
    rng = np.random.default_rng(0)
    H, I, Q = mc.hidden_size, mc.intermediate_size, mc.num_heads * mc.head_dim
    qkv = (mc.num_heads + 2 * mc.num_kv_heads) * mc.head_dim
    byts = {"QKV": qkv * H * 2, "O": Q * H * 2, "GU": 2 * I * H * 2, "DOWN": I * H * 2}
    for rows in a.rows:
        prompts = [rng.integers(300, 30000, size=a.ctx).tolist() for _ in range(rows)]
        sp = SamplingParams(temperature=0.2, max_tokens=a.steps, ignore_eos=True, seed=1)
        eng.generate(prompts, sp)
        torch.cuda.synchronize()
        # one more timed decode step set: time the graph replays
        t0 = time.perf_counter()
        eng.generate([p[:a.ctx] for p in prompts], SamplingParams(temperature=0.2, max_tokens=a.steps,
                                                                  ignore_eos=True, seed=2))
        torch.cuda.synchronize()
        tr = trace.cpu().numpy().astype(np.float64) / 100.0  # 100 MHz -> us
        st = stats.cpu().numpy().astype(np.float64)
        ends = tr[:, :, 1]
        crit = ends.max(axis=0)  # latest end per phase
        per = {k: [] for k in KINDS}
        for l in range(L):
            for j, k in enumerate(KINDS):
                p_ = 1 + 5 * l + j
                prev = p_ - 1 if p_ > 1 else None
                if prev is None or crit[prev] == 0:
                    continue
                per[k].append(crit[p_] - crit[prev])
        lm = 1 + 5 * L
        total = crit[lm] - crit[1] if crit[1] else 0
        print(f"== rows {rows}, ctx {a.ctx}: step span QKV0-end -> LM-end {total:.1f} us")
        for k in KINDS:
            v = np.array(per[k])
            sol = byts.get(k, 0) / 6.4e12 * 1e6
            print(f"  {k:5s} mean {v.mean():7.2f} us  p90 {np.percentile(v, 90):7.2f}  "
                  f"(weights at 6.4 TB/s: {sol:6.2f} us)")
        print(f"  LM    {crit[lm] - crit[lm - 1]:7.2f} us")
        lt = st[:, 1]
        if lt.sum() > 0:
            print(f"  loader FREE-wait {100 * st[:, 0].sum() / lt.sum():.1f} % of loader time; "
                  f"wave-0 FULL-wait {100 * st[:, 2].sum() / lt.sum():.1f} %; "
                  f"wave-0 poll {100 * st[:, 3].sum() / lt.sum():.1f} %")
        else:
            print("  register-streaming mode (no loader waves): wave-0 poll "
                  f"{st[:, 3].sum() / max(1, st.shape[0]) / 100.0:.1f} (x100 cycles per workgroup)")
        print(f"  err word {ops.decode_step_error(r.mk_sync, L)}")
    ops.set_decode_step_trace(None, None)


if __name__ == "__main__":
    main()
