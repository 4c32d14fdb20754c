"""End-to-end fan-out benchmark THROUGH the serving stack (BASELINE.json metric as the
reference measures it): the aiohttp llm-backend (serving/serve_llm.py), Agent A and five
Agent B servers, all in-process on 127.0.0.1 (testing/stack.py), driven by
``POST /task {"scenario": "agentic_parallel"}`` exactly like the reference's experiment
runner drives agent-a (reference agents/agent_a/server.py:441-648 ->
llm/serve_llm.py:731-942).

Per task: planning call -> 5 concurrent Agent B calls (each its own HTTP hop and LLM call) ->
final synthesis call.  Tokens/s = completion tokens reported by the backend's ``meta`` of
every LLM call / wall time; TTFT = each call's ``meta.queue_wait_s`` (submission -> first
token, exact - the dashboard histogram's lowest bucket is 0.5 s).  ``LLM_IGNORE_EOS=1`` makes
every call generate exactly ``LLM_MAX_TOKENS`` so runs are comparable with the in-process
engine bench (bench/fanout.py); the difference between the two numbers is the serving-layer
overhead (HTTP, JSON, tokenisation, asyncio hand-offs).
"""
from __future__ import annotations

import os
import statistics
import time

import httpx

from .fanout import TASKS


def run_e2e(engine, steps: int, warmup: int, fanout: int = 5, max_tokens: int = 512,
            log=None) -> dict:
    from ..agents.common.http import shared_ssl_context
    from ..testing.stack import Stack

    env = {"LLM_MAX_TOKENS": str(max_tokens), "LLM_IGNORE_EOS": "1", "LLM_TEMPERATURE": "0.2",
           "LLM_MAX_MODEL_LEN": str(engine.cfg.max_model_len),
           "AGENT_B_TIMEOUT_SECONDS": "600", "LLM_TIMEOUT_SECONDS": "600",
           "LOG_LLM_REQUESTS": "0"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)  # Settings() of the backend reads them at construction
    try:
        with Stack(engine=engine, n_agent_b=fanout) as st:
            url = st.agent_a_url + "/task"

            def one(i):
                t0 = time.perf_counter()
                r = httpx.post(url, json={"task": TASKS[i % len(TASKS)] + f" (run {i})",
                                          "scenario": "agentic_parallel",
                                          "agent_count": fanout}, timeout=1200,
                               verify=shared_ssl_context())
                r.raise_for_status()
                body = r.json()
                metas = [q.get("llm_meta") or {} for q in body.get("llm_requests", [])]
                return time.perf_counter() - t0, metas

            for i in range(warmup):
                dt, _ = one(i)
                if log:
                    log(f"e2e warmup {i}: {dt:.2f}s")
            t_start = time.perf_counter()
            runs = [one(warmup + i) for i in range(steps)]
            elapsed = time.perf_counter() - t_start
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    metas = [m for _, ms in runs for m in ms]
    tokens = sum(int(m.get("completion_tokens") or 0) for m in metas)
    ttfts = sorted(float(m["queue_wait_s"]) for m in metas if m.get("queue_wait_s") is not None)
    return {
        "tokens": tokens,
        "seconds": elapsed,
        "tokens_per_s": tokens / elapsed if elapsed > 0 else 0.0,
        "calls": len(metas),
        "p50_ttft_s": statistics.median(ttfts) if ttfts else None,
        "p95_ttft_s": ttfts[min(len(ttfts) - 1, int(0.95 * len(ttfts)))] if ttfts else None,
        "per_task_s": [round(d, 3) for d, _ in runs],
    }
