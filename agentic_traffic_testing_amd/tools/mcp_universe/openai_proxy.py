"""OpenAI-compatible ``POST /v1/chat/completions`` shim in front of the ``/chat`` backend.

Same contract as reference tools/mcp_universe/openai_proxy.py:43-165:

* messages are flattened to ``"[ROLE]\\n<content>\\n"`` blocks joined by blank lines
  (list-of-parts content keeps text parts only);
* the backend gets ``{"prompt": ..., "max_tokens"?}``; a non-200 backend answer or a
  connection error is a 502 with ``error`` / ``status`` / ``backend_body`` (500 chars);
* the reply is a ``chat.completion`` object with one ``stop`` choice; an empty backend
  output becomes ``"[Proxy] Local LLM backend returned empty output."``;
* ``GET /health`` and ``/ready`` report the backend URL; default port 8110.

Deliberate fix (SURVEY §2.1 T5 notes the reference always returns null usage): when the
backend's ``meta`` carries token counts (this backend's always does) they are reported in
``usage``; otherwise the fields stay null as before.  The proxy also keeps ONE pooled
aiohttp session instead of opening a new one per request.
"""
from __future__ import annotations

import argparse
import asyncio
import os
import time
import typing as t
import uuid

import aiohttp
from aiohttp import web

from . import DEFAULT_OPENAI_PROXY_HOST, DEFAULT_OPENAI_PROXY_PORT

BACKEND_URL_ENV = "LLM_SERVER_URL"
DEFAULT_BACKEND_URL = os.environ.get(BACKEND_URL_ENV, "http://llm-backend:8000/chat")
EMPTY_OUTPUT = "[Proxy] Local LLM backend returned empty output."
BACKEND_KEY = web.AppKey("backend_url", str)
SESSION_KEY = web.AppKey("session", aiohttp.ClientSession)


def flatten_messages(messages: t.Sequence[dict]) -> str:
    blocks = []
    for m in messages:
        content = m.get("content", "")
        if isinstance(content, list):
            texts = [b["text"] for b in content
                     if isinstance(b, dict) and b.get("type") == "text"
                     and isinstance(b.get("text"), str)]
            texts += [b for b in content if isinstance(b, str)]
            content = "\n".join(texts)
        elif not isinstance(content, str):
            content = str(content)
        blocks.append(f"[{str(m.get('role', 'user')).upper()}]\n{content}\n")
    return "\n".join(blocks).strip()


def _output_text(data) -> str:
    if isinstance(data, dict):
        if isinstance(data.get("output"), str):
            return data["output"]
        ch = data.get("choices")
        if isinstance(ch, list) and ch and isinstance(ch[0], dict):
            msg = ch[0].get("message") or {}
            if isinstance(msg.get("content"), str):
                return msg["content"]
    return ""


def _usage(data) -> dict:
    meta = data.get("meta") if isinstance(data, dict) else None
    if isinstance(meta, dict) and isinstance(meta.get("prompt_tokens"), int) \
            and isinstance(meta.get("completion_tokens"), int):
        p, c = meta["prompt_tokens"], meta["completion_tokens"]
        return {"prompt_tokens": p, "completion_tokens": c, "total_tokens": p + c}
    return {"prompt_tokens": None, "completion_tokens": None, "total_tokens": None}


async def handle_chat_completions(request: web.Request) -> web.Response:
    try:
        payload = await request.json()
    except Exception:
        return web.json_response({"error": "Invalid JSON body"}, status=400)
    if not isinstance(payload, dict):
        return web.json_response({"error": "Invalid JSON body"}, status=400)
    messages = payload.get("messages")
    if not isinstance(messages, list) or not messages:
        return web.json_response({"error": "Field 'messages' must be a non-empty list"},
                                 status=400)
    body: dict = {"prompt": flatten_messages(messages)}
    try:
        if payload.get("max_tokens") is not None:
            body["max_tokens"] = int(payload["max_tokens"])
    except (TypeError, ValueError):
        pass
    url = request.app[BACKEND_KEY]
    try:
        async with request.app[SESSION_KEY].post(url, json=body) as resp:
            if resp.status != 200:
                text = await resp.text()
                return web.json_response({"error": "Backend LLM request failed",
                                          "status": resp.status, "backend_body": text[:500]},
                                         status=502)
            data = await resp.json()
    except Exception as exc:
        return web.json_response({"error": f"Error calling local LLM backend: {exc}"},
                                 status=502)
    return web.json_response({
        "id": f"chatcmpl-{uuid.uuid4().hex[:24]}",
        "object": "chat.completion",
        "created": int(time.time()),
        "model": payload.get("model", "local-llm"),
        "choices": [{"index": 0,
                     "message": {"role": "assistant",
                                 "content": _output_text(data) or EMPTY_OUTPUT},
                     "finish_reason": "stop"}],
        "usage": _usage(data),
    })


def create_app(backend_url: str) -> web.Application:
    app = web.Application()
    app[BACKEND_KEY] = backend_url

    async def session_ctx(app_):
        timeout = aiohttp.ClientTimeout(total=float(os.environ.get("PROXY_TIMEOUT_S", "600")))
        app_[SESSION_KEY] = aiohttp.ClientSession(timeout=timeout)
        yield
        await app_[SESSION_KEY].close()

    app.cleanup_ctx.append(session_ctx)

    async def health(_):
        return web.json_response({"status": "ok", "backend_url": backend_url})

    app.router.add_post("/v1/chat/completions", handle_chat_completions)
    app.router.add_get("/health", health)
    app.router.add_get("/ready", health)
    return app


async def _serve(host: str, port: int, backend_url: str) -> None:
    runner = web.AppRunner(create_app(backend_url))
    await runner.setup()
    await web.TCPSite(runner, host, port).start()
    print(f"[openai-proxy] listening on http://{host}:{port} -> {backend_url}", flush=True)
    try:
        while True:
            await asyncio.sleep(3600)
    finally:
        await runner.cleanup()


def main(argv: list[str] | None = None) -> None:
    ap = argparse.ArgumentParser(description="OpenAI-compatible proxy to the local LLM backend")
    ap.add_argument("--host", default=DEFAULT_OPENAI_PROXY_HOST)
    ap.add_argument("--port", type=int, default=DEFAULT_OPENAI_PROXY_PORT)
    ap.add_argument("--backend-url", default=DEFAULT_BACKEND_URL,
                    help=f"/chat URL (default ${BACKEND_URL_ENV} or {DEFAULT_BACKEND_URL})")
    a = ap.parse_args(argv)
    try:
        asyncio.run(_serve(a.host, a.port, a.backend_url))
    except KeyboardInterrupt:
        print("[openai-proxy] stopped", flush=True)


if __name__ == "__main__":
    main()
