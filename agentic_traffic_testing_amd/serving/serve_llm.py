"""LLM backend HTTP server (``python -m llm.serve_llm``) on the MI355X-native engine.

API-compatible with the reference's aiohttp front end over vLLM (llm/serve_llm.py):

* ``POST /chat | /completion | /generate`` with ``{prompt|input, max_tokens?, request_id?,
  system_prompt?, skip_chat_template?}`` -> ``{"output", "meta": {request_id, latency_ms,
  queue_wait_s, prompt_tokens, completion_tokens, total_tokens, otel}}``; 400 on bad JSON /
  missing prompt, 503 before init, 500 ``Generation failed: ...`` (serve_llm.py:731-942);
* ``GET /health | /ready | /live`` -> ``{"status": "ok"}``; ``GET /metrics`` -> Prometheus
  text of the exact ``llm_*`` families (serving/metrics.py);
* the same stdout line protocol (``[llm] req=<id> START/PROGRESS/GENERATED/DONE/ERROR``),
  Llama-3 chat templating and head-keeping prompt truncation
  (``max(0, LLM_MAX_MODEL_LEN - max_new - LLM_PROMPT_SAFETY_MARGIN_TOKENS)``);
* the same CLI flags and env fallbacks (serve_llm.py:1050-1104).

Differences, by design: ``queue_wait_s`` is the engine-measured TTFT (submission -> first
token, incl. prefill, like the reference); ``completion_tokens`` is the engine's token count
(the reference re-tokenises the output text, serve_llm.py:881-882 - ``meta`` also carries
``completion_tokens_text`` for that definition); /health turns 503 when the engine loop has
stalled with work pending (watchdog).  Extra flags: ``--tensor-parallel-size``,
``--block-size``, ``--no-prefix-caching``, ``--no-graphs``, ``--load-format``.
"""
from __future__ import annotations

import argparse
import asyncio
import collections
import json
import os
import random
import sys
import time
import uuid

from aiohttp import web

from ..engine.sequence import SamplingParams
from ..engine.tokenizer import apply_chat_template
from ..utils import otel
from .metrics import CONTENT_TYPE_LATEST, LLMMetrics


def _env_bool(name: str, default: str) -> bool:
    return os.environ.get(name, default).lower() in ("1", "true", "yes", "on")


class Settings:
    def __init__(self):
        e = os.environ
        self.model = e.get("LLM_MODEL", "meta-llama/Llama-3.1-8B-Instruct")
        self.log_requests = _env_bool("LOG_LLM_REQUESTS", "")
        self.log_max_chars = int(e.get("LLM_LOG_MAX_CHARS", "500"))
        self.max_tokens = int(e.get("LLM_MAX_TOKENS", "512"))
        self.max_model_len_env = int(e.get("LLM_MAX_MODEL_LEN") or "0")
        self.margin = int(e.get("LLM_PROMPT_SAFETY_MARGIN_TOKENS", "128"))
        self.metrics_enabled = _env_bool("LLM_METRICS_ENABLED", "1")
        self.metrics_prefix = e.get("LLM_METRICS_PREFIX", "llm")
        self.apply_template = _env_bool("LLM_APPLY_CHAT_TEMPLATE", "1")
        self.temperature = float(e.get("LLM_TEMPERATURE", "0.2"))
        # benchmark knob: requests that do not say otherwise generate exactly max_tokens
        # (bench/e2e.py; random-init weights would otherwise stop at random EOS draws)
        self.ignore_eos = _env_bool("LLM_IGNORE_EOS", "")
        # benchmark knob: clamp every request's max_tokens (0 = off) - e.g. the AgentVerse
        # final synthesis asks for 4096 tokens, too long for a 70B stand-in run
        self.max_tokens_limit = int(e.get("LLM_MAX_TOKENS_LIMIT") or "0")
        self.watchdog_s = float(e.get("LLM_WATCHDOG_SECONDS", "120"))
        # fault injection: exercise the agents' error / timeout paths
        self.fault_fail_rate = float(e.get("LLM_FAULT_FAIL_RATE") or "0")
        self.fault_delay_s = float(e.get("LLM_FAULT_DELAY_MS") or "0") / 1000.0
        self.fault_step_delay_s = float(e.get("LLM_FAULT_STEP_DELAY_MS") or "0") / 1000.0
        self.fault_rng = random.Random(int(e.get("LLM_FAULT_SEED") or "0"))


class ServerState:
    def __init__(self, engine, async_engine, settings: Settings | None = None,
                 metrics: LLMMetrics | None = None, model_name: str = ""):
        self.engine = engine
        self.aengine = async_engine
        self.s = settings or Settings()
        self.metrics = metrics if metrics is not None else (
            LLMMetrics(self.s.metrics_prefix) if self.s.metrics_enabled else None)
        self.tracer = otel.get_tracer("llm-backend")
        self.inflight = 0
        self.peak_inflight = 0
        # per-request records of completed calls (bench/e2e.py reads them for workloads whose
        # clients do not see the backend meta, e.g. the OpenAI proxy)
        self.records: collections.deque = collections.deque(maxlen=200000)
        self.last_arrival: float | None = None
        self.model_name = model_name
        self.tok = engine.tokenizer if engine is not None else None

    def log(self, msg: str):
        print(msg, flush=True)

    # ----------------------------------------------------------------------------------
    def export_config(self):
        m, cfg = self.metrics, self.engine.cfg
        if m is None:
            return
        m.cfg_max_num_seqs.set(float(cfg.max_num_seqs))
        m.cfg_max_num_batched_tokens.set(float(cfg.max_num_batched_tokens))
        m.cfg_gpu_mem_util.set(float(cfg.gpu_memory_utilization))
        m.cfg_max_tokens.set(float(self.s.max_tokens))
        info = self.engine.kv_cache_info()
        m.set_kv(info["num_gpu_blocks"], info["block_size"], cfg.max_model_len)
        self.log(f"[llm-metrics] KV cache gauges set at startup: num_gpu_blocks="
                 f"{info['num_gpu_blocks']} block_size={info['block_size']} max_model_len="
                 f"{cfg.max_model_len} total_tokens={info['total_tokens']} est_max_concurrency="
                 f"{info['total_tokens'] // max(1, cfg.max_model_len)}")

    def on_step(self, stats, seconds: float):
        m = self.metrics
        if m is None:
            return
        m.batch_size.observe(stats.num_seqs)
        m.engine_steps.inc()
        m.engine_step_seconds.observe(seconds)

    def refresh_gauges(self):
        m = self.metrics
        if m is None or self.engine is None:
            return
        sch = self.engine.scheduler
        m.engine_running.set(len(sch.running))
        m.engine_waiting.set(len(sch.waiting))
        info = self.engine.kv_cache_info()
        m.kv_free_blocks.set(info["free_blocks"])
        m.prefix_hits.set(info["prefix_hits"])
        m.prefix_queries.set(info["prefix_queries"])
        if self.aengine is not None:
            m.heartbeat_age.set(max(0.0, time.monotonic() - self.aengine.heartbeat))


STATE_KEY = web.AppKey("state", ServerState)


def _log_prompt(st: ServerState, source: str, prompt: str):
    if not st.s.log_requests:
        return
    n = max(st.s.log_max_chars, 0)
    preview = prompt[:n] if n else ""
    suffix = "" if len(prompt) <= n else f"... [truncated {len(prompt) - n} chars]"
    st.log(f"[llm-request] source={source} prompt_len={len(prompt)} prompt={preview}{suffix}")


async def handle_health(request: web.Request) -> web.Response:
    st: ServerState = request.app[STATE_KEY]
    if st.aengine is not None and (not st.aengine.alive or st.aengine.stalled(st.s.watchdog_s)):
        return web.json_response({"status": "unhealthy", "reason": "engine loop stalled"},
                                 status=503)
    # kernel error word (prefill GEMM wait timed out -> tiles recomputed, outputs exact): the
    # GPU is shared or oversubscribed; still serving, so 200 with the reason attached
    # (words since the previous /health check: the runner clears them on read)
    runner = getattr(st.engine, "runner", None) if st.engine else None
    err = runner.take_kernel_error() if hasattr(runner, "take_kernel_error") else 0
    if err:
        return web.json_response({"status": "ok", "degraded": True,
                                  "kernel_error_word": int(err),
                                  "kernel_error_steps": int(runner.kernel_error_steps)})
    return web.json_response({"status": "ok"})


async def handle_metrics(request: web.Request) -> web.Response:
    st: ServerState = request.app[STATE_KEY]
    if st.metrics is None:
        return web.json_response({"error": "Metrics disabled"}, status=503)
    st.refresh_gauges()
    return web.Response(body=st.metrics.exposition(), headers={"Content-Type": CONTENT_TYPE_LATEST})


async def handle_chat(request: web.Request) -> web.Response:
    st: ServerState = request.app[STATE_KEY]
    if st.engine is None or st.aengine is None:
        return web.json_response({"error": "Backend not initialized"}, status=503)
    ctx = otel.extract(dict(request.headers))
    with st.tracer.start_as_current_span("llm.handle_request", context=ctx,
                                         kind=otel.SpanKind.SERVER) as span:
        start = time.monotonic()
        if st.last_arrival is not None and st.metrics is not None:
            st.metrics.interarrival.observe(start - st.last_arrival)
        st.last_arrival = start
        st.inflight += 1
        st.peak_inflight = max(st.peak_inflight, st.inflight)
        current_inflight = st.inflight
        if st.metrics:
            st.metrics.inflight.inc()
        span.set_attribute("app.path", request.path)

        def _leave():
            st.inflight -= 1
            if st.metrics:
                st.metrics.inflight.dec()
            return st.inflight

        try:
            data = await request.json()
            if not isinstance(data, dict):
                raise json.JSONDecodeError("not an object", "", 0)
        except (json.JSONDecodeError, UnicodeDecodeError, ValueError):
            _leave()
            return web.json_response({"error": "Invalid JSON"}, status=400)
        prompt = data.get("prompt") or data.get("input")
        if not isinstance(prompt, str) or not prompt:
            _leave()
            return web.json_response({"error": "Missing 'prompt' field"}, status=400)
        max_tokens = data.get("max_tokens")
        if max_tokens is not None and not isinstance(max_tokens, int):
            try:
                max_tokens = int(max_tokens)
            except (TypeError, ValueError):
                max_tokens = None
        rid = request.headers.get("X-Request-ID") or data.get("request_id")
        request_id = str(rid) if rid else str(uuid.uuid4())[:8]
        span.set_attribute("app.request_id", request_id)

        original = prompt
        skip = bool(data.get("skip_chat_template", False))
        templated = (not skip) and st.s.apply_template
        if templated:
            prompt = apply_chat_template(prompt, data.get("system_prompt"))
        ids = st.tok.encode(prompt)
        eff_new = max_tokens if max_tokens is not None else st.s.max_tokens
        if st.s.max_tokens_limit > 0:
            eff_new = min(eff_new, st.s.max_tokens_limit)
        truncated_tokens = None
        mml = st.s.max_model_len_env
        if mml > 0:
            keep = max(0, mml - eff_new - st.s.margin)
            if len(ids) > keep:
                truncated_tokens = len(ids) - keep
                st.log(f"[llm] req={request_id} PROMPT_TRUNCATED original_tokens={len(ids)} "
                       f"kept={keep} dropped={truncated_tokens}")
                ids = ids[:keep]
        span.set_attribute("app.prompt_length", len(original))
        span.set_attribute("app.formatted_prompt_length", len(prompt))
        span.set_attribute("app.chat_template_applied", templated)
        span.set_attribute("app.prompt_truncated", truncated_tokens is not None)
        if truncated_tokens is not None:
            span.set_attribute("app.prompt_truncated_tokens", int(truncated_tokens))
        if st.s.log_requests:
            span.set_attribute("app.prompt_preview", original[:200])
        _log_prompt(st, "http", original)
        tinfo = " (templated)" if templated else ""
        trunc = f" [TRUNCATED -{truncated_tokens}tok]" if truncated_tokens else ""
        st.log(f"[llm] req={request_id} START inflight={current_inflight} "
               f"prompt_len={len(original)}{tinfo}{trunc}")

        sp = SamplingParams(temperature=float(data.get("temperature", st.s.temperature)),
                            max_tokens=max(1, eff_new), ignore_eos=bool(data.get("ignore_eos", st.s.ignore_eos)),
                            seed=data.get("seed"))
        queue_wait = 0.0
        final = None
        try:
            if st.s.fault_delay_s > 0:
                await asyncio.sleep(st.s.fault_delay_s)
            if st.s.fault_fail_rate > 0 and st.s.fault_rng.random() < st.s.fault_fail_rate:
                span.set_attribute("app.fault_injected", True)
                raise RuntimeError("injected fault (LLM_FAULT_FAIL_RATE)")
            wait_span = st.tracer.start_span("llm.time_to_first_token")
            gen_span = None
            t_sub = time.monotonic()
            last_log = t_sub
            # burst-aware admission: the fan-out width Agent A announces (x-fanout, forwarded
            # by Agent B) groups the burst by its X-Task-ID
            burst = None
            fan = request.headers.get("x-fanout")
            task = request.headers.get("X-Task-ID")
            if fan and task:
                try:
                    burst = (task, int(fan))
                except ValueError:
                    burst = None
            async for out in st.aengine.generate(ids, sp, request_id, burst=burst):
                if gen_span is None:
                    queue_wait = time.monotonic() - t_sub
                    wait_span.set_attribute("llm_ttft_seconds", queue_wait)
                    wait_span.end()
                    gen_span = st.tracer.start_span("llm.generate")
                    gen_span.set_attribute("app.request_id", request_id)
                    t_first = time.monotonic()
                final = out
                now = time.monotonic()
                if now - last_log >= 2.0:
                    el = now - t_sub
                    st.log(f"[llm] req={request_id} PROGRESS tokens={len(out.token_ids)} "
                           f"speed={len(out.token_ids) / el if el > 0 else 0:.1f} tok/s")
                    last_log = now
            if wait_span.is_recording():
                wait_span.end()
            text = st.tok.decode(final.token_ids) if final is not None else ""
            el = time.monotonic() - t_sub
            ntok = len(final.token_ids) if final is not None else 0
            st.log(f"[llm] req={request_id} GENERATED tokens={ntok} time={el:.2f}s "
                   f"speed={ntok / el if el > 0 else 0:.1f} tok/s")
            _engine_spans(st, wait_span, gen_span, final)
            if gen_span is not None:
                gen_span.set_attribute("llm.generate_ms", int((time.monotonic() - t_first) * 1000))
                gen_span.end()
            prompt_tokens = len(ids)
            completion_tokens = ntok
            span.set_attribute("llm.prompt_tokens", prompt_tokens)
            span.set_attribute("llm.completion_tokens", completion_tokens)
            span.set_attribute("llm.total_tokens", prompt_tokens + completion_tokens)
        except Exception as exc:
            _leave()
            lat = time.monotonic() - start
            st.log(f"[llm] req={request_id} ERROR after {int(lat * 1000)}ms: {exc}")
            if st.metrics:
                st.metrics.record("error", lat, queue_wait, None, None)
            return web.json_response({"error": f"Generation failed: {exc}"}, status=500)

        remaining = _leave()
        lat = time.monotonic() - start
        latency_ms = int(lat * 1000)
        st.log(f"[llm] req={request_id} DONE latency={latency_ms}ms prompt={prompt_tokens} "
               f"completion={completion_tokens} remaining={remaining}")
        if st.metrics:
            st.metrics.record("success", lat, queue_wait, prompt_tokens, completion_tokens)
            st.metrics.ttft.observe(queue_wait)
        if st.s.log_requests:
            st.log(f"[llm-metrics] status=success latency_ms={latency_ms} prompt_tokens="
                   f"{prompt_tokens} completion_tokens={completion_tokens}")
        # engine-clock split of the TTFT: arrival -> first scheduled (hold + queue) -> first
        # token collected (prefill step); queue_wait_s minus engine_ttft_s is the hand-off from
        # the engine thread to this handler
        eng_ttft = final.ttft if final is not None else None
        sched = final.queue_wait if final is not None else None
        st.records.append({"t_end": time.time(), "queue_wait_s": queue_wait,
                           "prompt_tokens": prompt_tokens,
                           "completion_tokens": completion_tokens, "burst": burst,
                           "hold_s": st.aengine.hold_s.pop(request_id, 0.0),
                           "engine_ttft_s": eng_ttft, "sched_wait_s": sched})
        meta = {
            "request_id": request_id,
            "latency_ms": latency_ms,
            "queue_wait_s": round(queue_wait, 4),
            "prompt_tokens": prompt_tokens,
            "completion_tokens": completion_tokens,
            "total_tokens": prompt_tokens + completion_tokens,
            "otel": otel.span_metadata(span),
            "ttft_s": round(queue_wait, 6),
            "cached_prompt_tokens": final.cached_prompt_tokens if final else 0,
            "finish_reason": final.finish_reason if final else None,
            "completion_tokens_text": st.tok.count(text),
        }
        return web.json_response({"output": text, "meta": meta})


def _engine_spans(st: ServerState, wait_span, gen_span, final) -> None:
    """Engine-side child spans, recorded from the request's engine timestamps: queueing +
    prefill under ``llm.time_to_first_token`` (engine.prefill) and the decode steps under
    ``llm.generate`` (engine.decode_step, one span carrying the step count)."""
    if final is None or final.first_token_time is None:
        return
    off = time.time_ns() - time.perf_counter_ns()

    def ns(t: float) -> int:
        return int(t * 1e9) + off

    sched = final.first_scheduled_time or final.arrival_time
    sp = st.tracer.start_span("engine.prefill", context=otel.context_of(wait_span),
                              start_time=ns(sched))
    sp.set_attribute("llm.prompt_tokens", final.prompt_tokens)
    sp.set_attribute("llm.cached_prompt_tokens", final.cached_prompt_tokens)
    sp.set_attribute("engine.queue_ms", round((sched - final.arrival_time) * 1e3, 3))
    sp.end(end_time=ns(final.first_token_time))
    if gen_span is not None and final.finish_time is not None:
        steps = max(0, len(final.token_ids) - 1)
        dec = st.tracer.start_span("engine.decode_step", context=otel.context_of(gen_span),
                                   start_time=ns(final.first_token_time))
        dec.set_attribute("engine.decode_steps", steps)
        if steps:
            dec.set_attribute("engine.mean_step_ms",
                              round((final.finish_time - final.first_token_time) * 1e3 / steps, 4))
        dec.end(end_time=ns(final.finish_time))


def create_app(state: ServerState) -> web.Application:
    app = web.Application(client_max_size=64 * 1024 * 1024)
    app[STATE_KEY] = state
    app.router.add_get("/health", handle_health)
    app.router.add_get("/ready", handle_health)
    app.router.add_get("/live", handle_health)
    app.router.add_get("/metrics", handle_metrics)
    app.router.add_post("/chat", handle_chat)
    app.router.add_post("/completion", handle_chat)
    app.router.add_post("/generate", handle_chat)
    return app


def build_config(args):
    """EngineConfig from CLI args + env fallbacks (reference env knobs, compose defaults)."""
    from ..config import EngineConfig

    kw = dict(model=args.model)
    if args.max_model_len:
        kw["max_model_len"] = args.max_model_len
    if args.dtype:
        kw["dtype"] = args.dtype
    if args.max_num_seqs:
        kw["max_num_seqs"] = args.max_num_seqs
    if args.max_num_batched_tokens:
        kw["max_num_batched_tokens"] = args.max_num_batched_tokens
    if args.gpu_memory_utilization:
        kw["gpu_memory_utilization"] = args.gpu_memory_utilization
    if args.block_size:
        kw["block_size"] = args.block_size
    if args.tensor_parallel_size:
        kw["tensor_parallel_size"] = args.tensor_parallel_size
    kw["enable_prefix_caching"] = not args.no_prefix_caching
    kw["use_graphs"] = not args.no_graphs
    kw["load_format"] = args.load_format
    if args.device:
        kw["device"] = args.device
    if getattr(args, "quantization", None):
        kw["quantization"] = args.quantization
    if getattr(args, "burst_window_ms", None) is not None:
        kw["burst_window_ms"] = args.burst_window_ms
    if getattr(args, "burst_gap_ms", None) is not None:
        kw["burst_gap_ms"] = args.burst_gap_ms
    return EngineConfig.from_env(**kw)


def build_engine(args):
    """Build the (possibly tensor-parallel) engine from CLI args + env fallbacks."""
    from ..engine.llm_engine import LLMEngine

    cfg = build_config(args)
    if cfg.tensor_parallel_size > 1:
        from ..parallel.tp_engine import TPEngine

        # under torchrun (WORLD_SIZE set) the other ranks were started by the launcher
        external = int(os.environ.get("WORLD_SIZE", "1")) == cfg.tensor_parallel_size
        return TPEngine(cfg, external=external)
    eng = LLMEngine(cfg)
    eng.runner.capture_all(all_parts=True)
    return eng


async def run_server(args) -> None:
    from ..engine.async_engine import AsyncEngine

    print(f"[*] Initializing MI355X engine for {args.model}...", flush=True)
    t0 = time.time()
    eng = build_engine(args)
    state = ServerState(eng, None, model_name=args.model)
    aeng = AsyncEngine(eng, on_step=state.on_step)
    aeng.fault_injection_delay_s = state.s.fault_step_delay_s
    aeng.start()
    state.aengine = aeng
    state.export_config()
    app = create_app(state)
    runner = web.AppRunner(app, access_log=None)
    await runner.setup()
    site = web.TCPSite(runner, args.host, args.port)
    cfg = eng.cfg
    print("=" * 60)
    print("[*] MI355X serving engine ready")
    print(f"    Model: {args.model}")
    print(f"    URL: http://{args.host}:{args.port}")
    print(f"    max_num_seqs: {cfg.max_num_seqs}")
    print(f"    max_model_len: {cfg.max_model_len}")
    print(f"    tensor_parallel_size: {cfg.tensor_parallel_size}")
    print(f"    KV blocks: {eng.kv_cache_info()['num_gpu_blocks']} x {cfg.block_size} tokens")
    print(f"    init: {time.time() - t0:.1f}s")
    print("    Batching: ENABLED (continuous batching, chunked prefill, prefix caching)")
    print("=" * 60, flush=True)
    await site.start()
    try:
        while True:
            await asyncio.sleep(3600)
    except asyncio.CancelledError:
        pass
    finally:
        aeng.shutdown()
        await runner.cleanup()


def make_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="MI355X-native LLM backend for the agentic traffic testbed")
    p.add_argument("--model", default=os.environ.get("LLM_MODEL", "meta-llama/Llama-3.1-8B-Instruct"))
    p.add_argument("--host", default="0.0.0.0")
    p.add_argument("--port", type=int, default=8000)
    p.add_argument("--max-model-len", type=int, default=None)
    p.add_argument("--dtype", default=None)
    p.add_argument("--max-num-seqs", type=int, default=None)
    p.add_argument("--max-num-batched-tokens", type=int, default=None)
    p.add_argument("--gpu-memory-utilization", type=float, default=None)
    p.add_argument("--tensor-parallel-size", "--tp-size", type=int, default=None)
    p.add_argument("--quantization", "-q", choices=["fp8"],
                   default=os.environ.get("LLM_QUANTIZATION", "").lower() or None,
                   help="fp8 weight-only quantisation (OCP e4m3fn, per-row scales)")
    p.add_argument("--data-parallel-size", "--dp-size", type=int, default=1,
                   help="engine replicas, one per GPU, behind a router on --port "
                        "(parallel/dp_router.py)")
    p.add_argument("--block-size", type=int, default=None)
    p.add_argument("--no-prefix-caching", action="store_true")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--load-format", default="auto", choices=["auto", "dummy", "safetensors"])
    p.add_argument("--device", default=None)
    p.add_argument("--burst-window-ms", type=float, default=None,
                   help="burst-aware admission: hold an announced fan-out (x-fanout) up to this "
                        "long for its siblings (0 = FIFO admission, like vLLM)")
    p.add_argument("--burst-gap-ms", type=float, default=None,
                   help="... closing early once no sibling arrived for this long")
    p.add_argument("--config", default=None,
                   help="YAML file of EngineConfig keys (e.g. llm/config/llama-3.1-8b.yaml); "
                        "explicit flags win")
    return p


def apply_config_file(args):
    if not args.config:
        return args
    import yaml

    with open(args.config) as f:
        data = yaml.safe_load(f) or {}
    for key, val in data.items():
        attr = key.replace("-", "_")
        if attr == "enable_prefix_caching":
            if not val:
                args.no_prefix_caching = True
            continue
        if attr == "model" and args.model != make_parser().get_default("model"):
            continue
        if hasattr(args, attr) and getattr(args, attr) in (None, make_parser().get_default(attr)):
            setattr(args, attr, val)
    return args


def _tp_worker_rank(args) -> bool:
    """torchrun launch of a TP group: ranks > 0 replay rank 0's steps and never serve."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world <= 1 or rank == 0:
        return False
    from ..parallel.tp_engine import run_worker

    cfg = build_config(args)
    run_worker(cfg, rank, world, int(os.environ.get("MASTER_PORT", "29511")))
    return True


def main(argv=None) -> None:
    # the host driver only supports dmabuf IPC: without this, RCCL and the IPC all-reduce's
    # hipIpcGetMemHandle fail for TP > 1 (set before anything initialises HIP; compose and
    # the Dockerfile set it too, a bare `python -m llm.serve_llm` must not depend on them)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    args = apply_config_file(make_parser().parse_args(argv))
    if args.data_parallel_size and args.data_parallel_size > 1:
        from ..parallel import dp_router

        raw = list(sys.argv[1:] if argv is None else argv)
        fwd, skip = [], False
        for i, a in enumerate(raw):  # drop router-level flags, forward the engine flags
            if skip:
                skip = False
                continue
            if a in ("--data-parallel-size", "--dp-size", "--port", "--host"):
                skip = True
                continue
            if a.startswith(("--data-parallel-size=", "--dp-size=", "--port=", "--host=")):
                continue
            fwd.append(a)
        sys.exit(dp_router.main(["--host", args.host, "--port", str(args.port),
                                 "--num-replicas", str(args.data_parallel_size), *fwd]))
    if _tp_worker_rank(args):
        return
    try:
        asyncio.run(run_server(args))
    except KeyboardInterrupt:
        print("\n[*] Shutting down MI355X serving engine.")


if __name__ == "__main__":
    sys.exit(main())
