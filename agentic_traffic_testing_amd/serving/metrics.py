"""Prometheus metric families of the LLM backend.

Names, help texts, label sets and histogram buckets are the compatibility contract used by
the Grafana dashboard and the experiment scraper (reference llm/serve_llm.py:84-167,
SURVEY §5.5.1).  Additions (new names only, nothing renamed):

* ``llm_ttft_seconds`` - fine-bucket TTFT companion: the reference's TTFT histogram
  (``llm_queue_wait_seconds``) starts at 0.5 s and cannot resolve MI355X TTFTs;
* ``llm_batch_size`` is actually observed (one sample per engine step; declared but never
  observed in the reference, serve_llm.py:121-125);
* ``llm_engine_*`` gauges/counters: steps, running/waiting sequences, free KV blocks,
  prefix-cache hits, step latency, engine heartbeat age.
"""
from __future__ import annotations

from prometheus_client import (CollectorRegistry, Counter, Gauge, Histogram, PlatformCollector,
                               ProcessCollector, generate_latest)
from prometheus_client import CONTENT_TYPE_LATEST  # noqa: F401

LATENCY_BUCKETS = [0.5, 1.0, 2.5, 5.0, 10.0, 15.0, 20.0, 30.0, 45.0, 60.0, 90.0, 120.0, 180.0]
BATCH_BUCKETS = [1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 20, 32]
INTERARRIVAL_BUCKETS = [0.01, 0.05, 0.1, 0.25, 0.5, 1.0, 2.0, 5.0, 10.0, 30.0, 60.0]
TTFT_FINE_BUCKETS = [0.005, 0.01, 0.02, 0.03, 0.05, 0.075, 0.1, 0.15, 0.2, 0.3, 0.5, 0.75, 1.0,
                     2.5, 5.0, 10.0, 30.0]
STEP_BUCKETS = [0.001, 0.002, 0.003, 0.005, 0.0075, 0.01, 0.02, 0.05, 0.1, 0.25, 0.5, 1.0]


class LLMMetrics:
    def __init__(self, prefix: str = "llm", registry: CollectorRegistry | None = None,
                 process_collectors: bool = True):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        if process_collectors:
            ProcessCollector(registry=r)
            PlatformCollector(registry=r)
        p = prefix
        self.requests_total = Counter(f"{p}_requests_total", "Total LLM requests", ["status"],
                                      registry=r)
        self.request_latency = Histogram(f"{p}_request_latency_seconds",
                                         "End-to-end LLM request latency",
                                         buckets=LATENCY_BUCKETS, registry=r)
        self.queue_wait = Histogram(f"{p}_queue_wait_seconds",
                                    "Time spent waiting in vLLM queue", buckets=LATENCY_BUCKETS,
                                    registry=r)
        self.inflight = Gauge(f"{p}_inflight_requests", "In-flight LLM requests", registry=r)
        self.prompt_tokens = Counter(f"{p}_prompt_tokens_total", "Total prompt tokens",
                                     registry=r)
        self.completion_tokens = Counter(f"{p}_completion_tokens_total",
                                         "Total completion tokens", registry=r)
        self.batch_size = Histogram(f"{p}_batch_size", "Number of requests batched together",
                                    buckets=BATCH_BUCKETS, registry=r)
        self.cfg_max_num_seqs = Gauge(
            f"{p}_config_max_num_seqs",
            "Configured max_num_seqs (vLLM scheduler concurrency); -1 means default", registry=r)
        self.cfg_max_num_batched_tokens = Gauge(
            f"{p}_config_max_num_batched_tokens",
            "Configured max_num_batched_tokens (vLLM scheduler); -1 means default", registry=r)
        self.cfg_gpu_mem_util = Gauge(
            f"{p}_config_gpu_memory_utilization",
            "Configured GPU memory utilization target (0-1); -1 means default", registry=r)
        self.cfg_max_tokens = Gauge(f"{p}_config_max_tokens",
                                    "Configured max tokens per generation (LLM_MAX_TOKENS)",
                                    registry=r)
        self.kv_num_gpu_blocks = Gauge(
            f"{p}_kv_cache_num_gpu_blocks",
            "vLLM KV cache: number of GPU blocks allocated; -1 means unknown", registry=r)
        self.kv_block_size = Gauge(f"{p}_kv_cache_block_size_tokens",
                                   "vLLM KV cache: tokens per block; -1 means unknown",
                                   registry=r)
        self.kv_total_tokens = Gauge(
            f"{p}_kv_cache_total_tokens",
            "vLLM KV cache: total tokens available in GPU KV cache (num_gpu_blocks * "
            "block_size); -1 means unknown", registry=r)
        self.kv_est_max_conc = Gauge(
            f"{p}_kv_cache_est_max_concurrency_at_max_model_len",
            "Estimated max concurrent sequences limited by KV cache at max_model_len; -1 means "
            "unknown", registry=r)
        self.computed_max_conc = Gauge(
            f"{p}_computed_max_concurrency",
            "KV-cache-derived max concurrency: num_gpu_blocks * block_size / max_model_len "
            "(matches the 'Maximum concurrency for X tokens' line vLLM logs at startup)",
            registry=r)
        self.interarrival = Histogram(f"{p}_interarrival_seconds",
                                      "Time between consecutive LLM request arrivals",
                                      buckets=INTERARRIVAL_BUCKETS, registry=r)
        # ---- additions (MI355X engine) -------------------------------------------------
        self.ttft = Histogram(f"{p}_ttft_seconds",
                              "Time to first token (fine buckets; same quantity as "
                              f"{p}_queue_wait_seconds)", buckets=TTFT_FINE_BUCKETS, registry=r)
        self.engine_steps = Counter(f"{p}_engine_steps_total", "Engine forward steps", registry=r)
        self.engine_step_seconds = Histogram(f"{p}_engine_step_seconds",
                                             "Engine step (forward + sample) wall time",
                                             buckets=STEP_BUCKETS, registry=r)
        self.engine_running = Gauge(f"{p}_engine_running_sequences", "Sequences running",
                                    registry=r)
        self.engine_waiting = Gauge(f"{p}_engine_waiting_sequences", "Sequences queued",
                                    registry=r)
        self.kv_free_blocks = Gauge(f"{p}_kv_cache_free_blocks", "Free + evictable KV blocks",
                                    registry=r)
        self.prefix_hits = Gauge(f"{p}_prefix_cache_hit_blocks", "Prefix-cache block hits",
                                 registry=r)
        self.prefix_queries = Gauge(f"{p}_prefix_cache_query_blocks",
                                    "Prefix-cache block lookups", registry=r)
        self.heartbeat_age = Gauge(f"{p}_engine_heartbeat_age_seconds",
                                   "Seconds since the engine loop last made progress",
                                   registry=r)

    def record(self, status: str, latency_s: float, queue_wait_s: float, prompt_tokens,
               completion_tokens):
        """The reference's _record_metrics (serve_llm.py:191-206)."""
        self.requests_total.labels(status=status).inc()
        self.request_latency.observe(latency_s)
        self.queue_wait.observe(queue_wait_s)
        if prompt_tokens is not None:
            self.prompt_tokens.inc(prompt_tokens)
        if completion_tokens is not None:
            self.completion_tokens.inc(completion_tokens)

    def set_kv(self, num_gpu_blocks: int, block_size: int, max_model_len: int):
        """The reference's _update_kv_cache_gauges (serve_llm.py:209-221)."""
        self.kv_num_gpu_blocks.set(float(num_gpu_blocks))
        self.kv_block_size.set(float(block_size))
        total = num_gpu_blocks * block_size
        self.kv_total_tokens.set(float(total))
        if max_model_len > 0:
            self.kv_est_max_conc.set(float(total // max_model_len))
            self.computed_max_conc.set(total / max_model_len)

    def exposition(self) -> bytes:
        return generate_latest(self.registry)
