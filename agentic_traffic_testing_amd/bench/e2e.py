"""End-to-end benchmarks THROUGH the serving stack: the aiohttp llm-backend
(serving/serve_llm.py), Agent A and N Agent B servers, all in-process on 127.0.0.1
(testing/stack.py), driven over HTTP exactly like the reference's clients drive them.

Workloads (``--workload``):

* ``agentic_parallel`` (the BASELINE.json headline, config 1-3): ``POST /task
  {"scenario": "agentic_parallel"}`` (reference agents/agent_a/server.py:441-648): planning
  call -> N concurrent Agent B calls (each its own HTTP hop and LLM call) -> final synthesis.
* ``agentverse`` (config 4): ``POST /agentverse`` with ``max_iterations`` 3,
  ``success_threshold`` 90 and ``stream: false``, as the reference experiment runner sends it
  (scripts/experiment/run_experiment.sh:346-395): recruitment, horizontal discussion or
  vertical review (reviewers in parallel), parallel execution on the Agent B replicas,
  evaluation, final synthesis (reference agents/agent_a/orchestrator.py:1859-2009).  Random-init
  weights parse nothing, so ``AGENTVERSE_ORACLE=1`` substitutes seeded recruitment / score
  decisions after each real LLM call (the request stream keeps its full length).
* ``proxy`` (config 5's MCP-Universe path): N concurrent agents run multi-turn tool-using
  conversations through the OpenAI-compatible proxy (tools/mcp_universe/openai_proxy.py ->
  ``/v1/chat/completions`` -> llm-backend ``/chat``; reference
  tools/mcp_universe/openai_proxy.py:67-164): every turn sends the growing message history
  (system + task + assistant replies + synthetic tool results).

Metrics come from the backend's own per-request records (``ServerState.records``: the meta it
returns - completion tokens, ``queue_wait_s`` = submission -> first token), so every workload
is counted the same way, including the proxy whose responses do not carry the meta:
tokens/s = completion tokens / wall time of the timed tasks, TTFT p50 / p95, LLM calls per
workflow and the peak number of in-flight backend requests.  ``LLM_IGNORE_EOS=1`` makes calls
generate their full budget (random weights would stop at random EOS draws).
"""
from __future__ import annotations

import asyncio
import os
import statistics
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import httpx

from .fanout import TASKS

WORKLOADS = ("agentic_parallel", "agentverse", "proxy")

PROXY_SYSTEM = ("You are an autonomous agent with access to MCP tools: get_stock_price(symbol), "
                "calculate_portfolio_value(holdings), geocode_location(name), "
                "calculate_distance(a, b), execute_python_code(code).  Think step by step; "
                "call one tool per turn as JSON {\"tool\": ..., \"args\": ...}; answer when done.")


class _ProxyThread:
    """The OpenAI-compatible proxy on its own event loop (ephemeral port)."""

    def __init__(self, backend_url: str):
        from aiohttp import web

        from ..tools.mcp_universe.openai_proxy import create_app

        self._loop = asyncio.new_event_loop()
        self._ready = threading.Event()
        self.port = 0

        def run():
            asyncio.set_event_loop(self._loop)
            runner = web.AppRunner(create_app(backend_url), access_log=None)
            self._loop.run_until_complete(runner.setup())
            site = web.TCPSite(runner, "127.0.0.1", 0)
            self._loop.run_until_complete(site.start())
            self.port = site._server.sockets[0].getsockname()[1]
            self._runner = runner
            self._ready.set()
            self._loop.run_forever()

        self._t = threading.Thread(target=run, daemon=True, name="openai-proxy")
        self._t.start()
        if not self._ready.wait(30):
            raise RuntimeError("proxy did not start")

    @property
    def url(self) -> str:
        return f"http://127.0.0.1:{self.port}/v1/chat/completions"

    def stop(self):
        fut = asyncio.run_coroutine_threadsafe(self._runner.cleanup(), self._loop)
        try:
            fut.result(10)
        except Exception:
            pass
        self._loop.call_soon_threadsafe(self._loop.stop)


def _proxy_session(url: str, idx: int, turns: int, max_tokens: int) -> int:
    """One MCP-Universe-style agent: ``turns`` chat completions over a growing history."""
    msgs = [{"role": "system", "content": PROXY_SYSTEM},
            {"role": "user", "content": TASKS[idx % len(TASKS)]}]
    calls = 0
    with httpx.Client(timeout=1200) as c:
        for t in range(turns):
            r = c.post(url, json={"model": "local", "messages": msgs, "max_tokens": max_tokens,
                                  "temperature": 0.2})
            r.raise_for_status()
            reply = r.json()["choices"][0]["message"]["content"] or ""
            calls += 1
            msgs.append({"role": "assistant", "content": reply[:1200]})
            msgs.append({"role": "user", "content": f"[tool result {t}] "
                         f"{{\"status\": \"ok\", \"value\": {100 + 7 * t + idx}}}"})
    return calls


def run_e2e(engine, steps: int, warmup: int, fanout: int = 5, max_tokens: int = 512,
            log=None, workload: str = "agentic_parallel", max_tokens_limit: int = 0,
            proxy_turns: int = 4, arrival_skew_ms: float = 0.0) -> dict:
    from ..agents.common.http import shared_ssl_context
    from ..testing.stack import Stack

    if workload not in WORKLOADS:
        raise ValueError(f"unknown workload {workload!r}")
    env = {"LLM_MAX_TOKENS": str(max_tokens), "LLM_IGNORE_EOS": "1", "LLM_TEMPERATURE": "0.2",
           "LLM_MAX_MODEL_LEN": str(engine.cfg.max_model_len),
           "AGENT_B_TIMEOUT_SECONDS": "1200", "LLM_TIMEOUT_SECONDS": "1200",
           "AGENTVERSE_LLM_TIMEOUT_SECONDS": "1200", "LOG_LLM_REQUESTS": "0",
           "LLM_MAX_TOKENS_LIMIT": str(max_tokens_limit), "AGENTVERSE_ORACLE": "1",
           # Agent A staggers fan-out worker i by i * ms (L7 arrival skew, burst experiments)
           "AGENT_FANOUT_STAGGER_MS": str(arrival_skew_ms)}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)  # Settings() of the backend reads them at construction
    proxy = None
    try:
        with Stack(engine=engine, n_agent_b=fanout) as st:
            state = st.llm.state
            if workload == "proxy":
                proxy = _ProxyThread(st.llm.url + "/chat")

            def one(i):
                t0 = time.perf_counter()
                if workload == "agentic_parallel":
                    r = httpx.post(st.agent_a_url + "/task",
                                   json={"task": TASKS[i % len(TASKS)] + f" (run {i})",
                                         "scenario": "agentic_parallel", "agent_count": fanout},
                                   timeout=3600, verify=shared_ssl_context())
                    r.raise_for_status()
                elif workload == "agentverse":
                    r = httpx.post(st.agent_a_url + "/agentverse",
                                   json={"task": TASKS[i % len(TASKS)] + f" (run {i})",
                                         "max_iterations": 3, "success_threshold": 90,
                                         "stream": False}, timeout=7200,
                                   verify=shared_ssl_context())
                    r.raise_for_status()
                else:
                    with ThreadPoolExecutor(max_workers=fanout) as pool:
                        list(pool.map(lambda k: _proxy_session(proxy.url, i * fanout + k,
                                                               proxy_turns, max_tokens),
                                      range(fanout)))
                return time.perf_counter() - t0

            for i in range(warmup):
                dt = one(i)
                if log:
                    log(f"e2e {workload} warmup {i}: {dt:.2f}s")
            state.records.clear()
            state.peak_inflight = state.inflight
            t_start = time.perf_counter()
            per_task = [one(warmup + i) for i in range(steps)]
            elapsed = time.perf_counter() - t_start
            recs = list(state.records)
            peak = state.peak_inflight
            coalesced = st.llm.aengine.bursts_coalesced
    finally:
        if proxy is not None:
            proxy.stop()
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    tokens = sum(int(r["completion_tokens"]) for r in recs)
    ttfts = sorted(float(r["queue_wait_s"]) for r in recs)

    def med(xs):
        xs = [float(x) for x in xs]
        return round(statistics.median(xs), 4) if xs else None

    # TTFT split: fan-out (burst) requests vs solo calls, and the part of a burst request's
    # TTFT spent held for its siblings (burst-aware admission)
    breakdown = {
        "burst_calls": sum(1 for r in recs if r.get("burst")),
        "p50_ttft_burst_s": med(r["queue_wait_s"] for r in recs if r.get("burst")),
        "p50_ttft_solo_s": med(r["queue_wait_s"] for r in recs if not r.get("burst")),
        "p50_hold_burst_s": med(r.get("hold_s", 0.0) for r in recs if r.get("burst")),
        # engine clock: arrival -> scheduled (INCLUDES the hold), scheduled -> first token;
        # the rest of the HTTP TTFT is the engine-thread -> event-loop hand-off.  The parts
        # add up as ttft = sched_wait + prefill + handoff, with sched_wait = hold + the wait
        # between the burst's release and its first engine step (p50_admit_wait_burst_s)
        "p50_sched_wait_burst_s": med(r["sched_wait_s"] for r in recs
                                      if r.get("burst") and r.get("sched_wait_s") is not None),
        "p50_admit_wait_burst_s": med(max(0.0, r["sched_wait_s"] - r.get("hold_s", 0.0))
                                      for r in recs
                                      if r.get("burst") and r.get("sched_wait_s") is not None),
        "p50_prefill_burst_s": med(r["engine_ttft_s"] - r["sched_wait_s"] for r in recs
                                   if r.get("burst") and r.get("engine_ttft_s") is not None
                                   and r.get("sched_wait_s") is not None),
        "p50_handoff_s": med(r["queue_wait_s"] - r["engine_ttft_s"] for r in recs
                             if r.get("engine_ttft_s") is not None),
    }
    return {
        "workload": workload,
        "tokens": tokens,
        "seconds": elapsed,
        "tokens_per_s": tokens / elapsed if elapsed > 0 else 0.0,
        "calls": len(recs),
        "calls_per_workflow": round(len(recs) / max(1, steps), 2),
        "peak_inflight": peak,
        "bursts_coalesced": coalesced,
        "p50_ttft_s": statistics.median(ttfts) if ttfts else None,
        "p95_ttft_s": ttfts[min(len(ttfts) - 1, int(0.95 * len(ttfts)))] if ttfts else None,
        "per_task_s": [round(d, 3) for d in per_task],
        "ttft_breakdown": breakdown,
    }
