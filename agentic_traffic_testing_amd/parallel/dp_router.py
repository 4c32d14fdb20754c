"""Data-parallel engine replicas behind one ``llm-backend:8000`` API.

The reference runs exactly one backend on one GPU (infra/docker-compose.yml:46-52).  On an
8 x MI355X node the 8B model is weight-bandwidth-bound at small batch on each GPU, so the
aggregate tokens/s of a fan-out workload scales best with one engine replica per GPU (the
bench's ``dp`` mode measures exactly that).  This router keeps the serving contract:

* ``POST /chat|/completion|/generate`` are forwarded verbatim (headers ``X-Request-ID``,
  ``X-Task-ID``, ``traceparent`` included) to one replica and its JSON answer returned;
* placement policy ``least_loaded`` (default: fewest in-flight requests, ties round-robin),
  ``round_robin``, or ``task_affinity`` (requests sharing ``X-Task-ID`` go to the same
  replica while it is not more than ``affinity_slack`` requests busier than the least
  loaded one - AgentVerse / multi-hop calls of one task share prompt prefixes, so affinity
  turns them into prefix-cache hits on that replica);
* the router records the ``llm_*`` contract metrics itself (request counts, latency, TTFT
  from the replica's ``meta.queue_wait_s``, tokens, interarrival, in-flight), so Prometheus
  and the dashboard see one logical backend; ``/metrics`` also exposes per-replica in-flight
  and request counters (``llm_router_*``);
* ``/health`` is 200 while at least one replica answers its own ``/health``; unhealthy
  replicas are skipped until a background probe sees them recover.

``spawn_replicas(n, ...)`` starts ``n`` ``serve_llm`` processes, replica i on GPU i
(``HIP_VISIBLE_DEVICES=i``, port ``base_port + i``); the router itself never touches a GPU.
"""
from __future__ import annotations

import argparse
import asyncio
import itertools
import os
import subprocess
import sys
import time

import aiohttp
from aiohttp import web
from prometheus_client import Counter, Gauge

from ..serving.metrics import CONTENT_TYPE_LATEST, LLMMetrics

FORWARD_HEADERS = ("X-Request-ID", "X-Task-ID", "traceparent", "tracestate", "x-agent-index")
STATE = web.AppKey("router", object)


class Replica:
    def __init__(self, url: str):
        self.url = url.rstrip("/")
        self.inflight = 0
        self.healthy = True
        self.requests = 0
        self.errors = 0


class Router:
    def __init__(self, backends: list[str], policy: str = "least_loaded",
                 affinity_slack: int = 2, timeout_s: float = 600.0,
                 metrics: LLMMetrics | None = None):
        if not backends:
            raise ValueError("no backends")
        self.replicas = [Replica(u) for u in backends]
        self.policy = policy
        self.affinity_slack = affinity_slack
        self.timeout_s = timeout_s
        self._rr = itertools.count()
        self.affinity: dict[str, Replica] = {}
        self.metrics = metrics or LLMMetrics()
        r = self.metrics.registry
        self.rep_inflight = Gauge("llm_router_replica_inflight", "In-flight requests per replica",
                                  ["replica"], registry=r)
        self.rep_requests = Counter("llm_router_replica_requests_total",
                                    "Requests routed per replica", ["replica", "status"],
                                    registry=r)
        self.rep_healthy = Gauge("llm_router_replica_healthy", "Replica health (1/0)",
                                 ["replica"], registry=r)
        self.last_arrival: float | None = None
        self.session: aiohttp.ClientSession | None = None

    # -- placement --------------------------------------------------------------------
    def pick(self, task_id: str | None = None) -> Replica:
        live = [r for r in self.replicas if r.healthy] or self.replicas
        least = min(r.inflight for r in live)
        if self.policy == "task_affinity" and task_id:
            r = self.affinity.get(task_id)
            if r is not None and r in live and r.inflight <= least + self.affinity_slack:
                return r
        if self.policy == "round_robin":
            chosen = live[next(self._rr) % len(live)]
        else:
            cands = [r for r in live if r.inflight == least]
            chosen = cands[next(self._rr) % len(cands)]
        if task_id and self.policy == "task_affinity":
            if len(self.affinity) > 100_000:
                self.affinity.clear()
            self.affinity[task_id] = chosen
        return chosen

    # -- request path -------------------------------------------------------------------
    async def forward(self, request: web.Request) -> web.Response:
        t0 = time.perf_counter()
        now = time.monotonic()
        if self.last_arrival is not None:
            self.metrics.interarrival.observe(now - self.last_arrival)
        self.last_arrival = now
        body = await request.read()
        hdrs = {h: request.headers[h] for h in FORWARD_HEADERS if h in request.headers}
        hdrs["Content-Type"] = "application/json"
        rep = self.pick(request.headers.get("X-Task-ID"))
        rep.inflight += 1
        self.metrics.inflight.inc()
        self.rep_inflight.labels(rep.url).set(rep.inflight)
        status, data, text = 502, None, ""
        try:
            async with self.session.post(rep.url + request.path, data=body, headers=hdrs) as resp:
                status = resp.status
                text = await resp.text()
                try:
                    data = await resp.json(content_type=None)
                except (ValueError, aiohttp.ContentTypeError):
                    data = None
        except (aiohttp.ClientError, asyncio.TimeoutError) as e:
            rep.healthy = False
            text = f'{{"error": "replica {rep.url} failed: {type(e).__name__}"}}'
        finally:
            rep.inflight -= 1
            self.metrics.inflight.dec()
            self.rep_inflight.labels(rep.url).set(rep.inflight)
        ok = status == 200 and isinstance(data, dict) and "output" in data
        rep.requests += 1
        rep.errors += 0 if ok else 1
        self.rep_requests.labels(rep.url, "success" if ok else "error").inc()
        if status not in (400,):  # client errors are not backend outcomes in the reference
            meta = data.get("meta", {}) if ok else {}
            self.metrics.record("success" if ok else "error", time.perf_counter() - t0,
                                float(meta.get("queue_wait_s") or 0.0) if ok else 0.0,
                                meta.get("prompt_tokens") if ok else None,
                                meta.get("completion_tokens") if ok else None)
            if ok and meta.get("queue_wait_s") is not None:
                self.metrics.ttft.observe(float(meta["queue_wait_s"]))
        return web.Response(status=status, text=text, content_type="application/json")

    async def probe(self, interval_s: float = 2.0):
        while True:
            for r in self.replicas:
                try:
                    async with self.session.get(r.url + "/health",
                                                timeout=aiohttp.ClientTimeout(total=2)) as resp:
                        r.healthy = resp.status == 200
                except (aiohttp.ClientError, asyncio.TimeoutError):
                    r.healthy = False
                self.rep_healthy.labels(r.url).set(1 if r.healthy else 0)
            await asyncio.sleep(interval_s)


def create_app(router: Router, probe_interval_s: float = 2.0) -> web.Application:
    app = web.Application(client_max_size=64 * 1024 * 1024)
    app[STATE] = router

    async def ctx(app_):
        router.session = aiohttp.ClientSession(
            timeout=aiohttp.ClientTimeout(total=router.timeout_s),
            connector=aiohttp.TCPConnector(limit=0))
        task = asyncio.ensure_future(router.probe(probe_interval_s))
        yield
        task.cancel()
        await router.session.close()

    app.cleanup_ctx.append(ctx)

    async def health(_):
        ok = any(r.healthy for r in router.replicas)
        return web.json_response({"status": "ok" if ok else "unavailable",
                                  "replicas": [{"url": r.url, "healthy": r.healthy,
                                                "inflight": r.inflight} for r in router.replicas]},
                                 status=200 if ok else 503)

    async def metrics(_):
        return web.Response(body=router.metrics.exposition(),
                            headers={"Content-Type": CONTENT_TYPE_LATEST})

    for path in ("/chat", "/completion", "/generate"):
        app.router.add_post(path, router.forward)
    for path in ("/health", "/ready", "/live"):
        app.router.add_get(path, health)
    app.router.add_get("/metrics", metrics)
    return app


def spawn_replicas(n: int, base_port: int, serve_args: list[str], log_dir: str = "logs",
                   gpus: list[int] | None = None):
    """Start n serve_llm processes, replica i pinned to GPU ``gpus[i]`` (default: GPU i;
    several replicas may share a GPU, e.g. the single-GPU rehearsal test)."""
    os.makedirs(log_dir, exist_ok=True)
    gpus = list(range(n)) if gpus is None else gpus
    procs = []
    for i in range(n):
        env = dict(os.environ, HIP_VISIBLE_DEVICES=str(gpus[i]), HSA_ENABLE_IPC_MODE_LEGACY="0")
        # the child inherits its own copy of the log descriptor; the parent's closes here
        with open(os.path.join(log_dir, f"llm_replica_{i}.log"), "a") as log:
            procs.append(subprocess.Popen(
                [sys.executable, "-m", "agentic_traffic_testing_amd.serving.serve_llm",
                 "--host", "127.0.0.1", "--port", str(base_port + i), *serve_args],
                env=env, stdout=log, stderr=subprocess.STDOUT))
    return procs


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Data-parallel router over LLM backend replicas")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--backends", default=os.environ.get("LLM_BACKEND_URLS", ""),
                    help="comma-separated replica base URLs (http://host:port)")
    ap.add_argument("--num-replicas", type=int, default=0,
                    help="spawn this many local replicas (one per GPU) instead of --backends")
    ap.add_argument("--base-port", type=int, default=8001)
    ap.add_argument("--policy", default="least_loaded",
                    choices=["least_loaded", "round_robin", "task_affinity"])
    a, serve_args = ap.parse_known_args(argv)
    procs = []
    if a.num_replicas > 0:
        procs = spawn_replicas(a.num_replicas, a.base_port, serve_args)
        backends = [f"http://127.0.0.1:{a.base_port + i}" for i in range(a.num_replicas)]
    else:
        backends = [u for u in a.backends.split(",") if u.strip()]
    router = Router(backends, a.policy)
    print(f"[*] DP router on http://{a.host}:{a.port} -> {backends} ({a.policy})", flush=True)
    try:
        web.run_app(create_app(router), host=a.host, port=a.port, access_log=None)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(30)
            except subprocess.TimeoutExpired:
                p.kill()
    return 0


if __name__ == "__main__":
    sys.exit(main())
