"""In-process testbed stacks for tests, demos and the CPU plumbing config.

``LLMBackendThread`` runs the real aiohttp LLM backend (serving/serve_llm.py) with its
engine on a background event loop; ``start_agent_b`` / ``start_agent_a`` run the real
ThreadingHTTPServer agents on ephemeral ports.  ``Stack`` wires them together the way the
compose files do (LLM_SERVER_URL, AGENT_B_URLS) so the whole L7/L8 request flow - HTTP,
headers, trace propagation, telemetry files - is exercised without Docker.
"""
from __future__ import annotations

import asyncio
import os
import threading
import time

from aiohttp import web


class LLMBackendThread:
    def __init__(self, engine, host: str = "127.0.0.1", port: int = 0, settings=None):
        from ..engine.async_engine import AsyncEngine
        from ..serving.serve_llm import ServerState, create_app

        self.engine = engine
        self.state = ServerState(engine, None, settings=settings)
        self.aengine = AsyncEngine(engine, on_step=self.state.on_step).start()
        self.state.aengine = self.aengine
        self.state.export_config()
        self.app = create_app(self.state)
        self.host, self.port = host, port
        self._loop = asyncio.new_event_loop()
        self._ready = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True, name="llm-backend")
        self._t.start()
        if not self._ready.wait(30):
            raise RuntimeError("LLM backend did not start")

    def _run(self):
        asyncio.set_event_loop(self._loop)
        runner = web.AppRunner(self.app, access_log=None)
        self._loop.run_until_complete(runner.setup())
        site = web.TCPSite(runner, self.host, self.port)
        self._loop.run_until_complete(site.start())
        self.port = site._server.sockets[0].getsockname()[1]
        self._runner = runner
        self._ready.set()
        self._loop.run_forever()

    @property
    def url(self) -> str:
        return f"http://{self.host}:{self.port}"

    def stop(self):
        self.aengine.shutdown()

        async def _cleanup():
            await self._runner.cleanup()

        fut = asyncio.run_coroutine_threadsafe(_cleanup(), self._loop)
        try:
            fut.result(10)
        except Exception:
            pass
        self._loop.call_soon_threadsafe(self._loop.stop)


def cpu_engine(model: str = "tiny", max_model_len: int = 1024, num_kv_blocks: int = 512,
               max_num_seqs: int = 8, max_num_batched_tokens: int = 1024):
    from ..config import EngineConfig
    from ..engine.llm_engine import LLMEngine

    cfg = EngineConfig(model=model, device="cpu", max_model_len=max_model_len,
                       num_kv_blocks=num_kv_blocks, max_num_seqs=max_num_seqs,
                       max_num_batched_tokens=max_num_batched_tokens, use_graphs=False)
    return LLMEngine(cfg)


class Stack:
    """LLM backend + N Agent B + Agent A, all in-process on 127.0.0.1."""

    def __init__(self, engine=None, n_agent_b: int = 5, log_dir: str | None = None,
                 env: dict | None = None):
        self._old_env = {}
        self.log_dir = log_dir
        if log_dir:
            self._set_env("TELEMETRY_LOG_DIR", log_dir)
            self._set_env("METRICS_LOG_DIR", log_dir)
            self._set_env("AGENTVERSE_LOG_DIR", log_dir)
        self._set_env("OTEL_SDK_DISABLED", "true")
        for k, v in (env or {}).items():
            self._set_env(k, v)
        self.llm = LLMBackendThread(engine or cpu_engine())
        self._set_env("LLM_SERVER_URL", self.llm.url + "/chat")
        from ..agents.agent_a.server import AgentAHandler
        from ..agents.agent_b.server import AgentBHandler
        from ..agents.common.http import start_background

        self.agent_b = [start_background(AgentBHandler) for _ in range(n_agent_b)]
        urls = [u + "/subtask" for _, u in self.agent_b]
        self._set_env("AGENT_B_URLS", ",".join(urls))
        self._set_env("AGENT_B_URL", urls[0])
        self.agent_a, self.agent_a_url = start_background(AgentAHandler)

    def _set_env(self, k, v):
        self._old_env.setdefault(k, os.environ.get(k))
        os.environ[k] = str(v)

    def stop(self):
        self.agent_a.shutdown()
        for s, _ in self.agent_b:
            s.shutdown()
        self.llm.stop()
        for k, v in self._old_env.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.stop()


def wait_http(url: str, timeout: float = 30.0) -> bool:
    import httpx

    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if httpx.get(url, timeout=2).status_code < 500:
                return True
        except Exception:
            time.sleep(0.2)
    return False
