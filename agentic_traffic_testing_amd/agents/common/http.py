"""HTTP plumbing shared by the agent services.

Traffic signature matters in this testbed: the agents are
``ThreadingHTTPServer`` processes (one thread per request, HTTP/1.0 -> the server closes
each connection), and the Agent A / Agent B helper calls use a *new* TCP connection per
call (module-level ``httpx.post``, reference agents/agent_a/main.py:26-68), while the
AgentVerse orchestrator keeps one persistent client (orchestrator.py:214).  Both client
styles are provided so each call site keeps its connection behaviour (SYN counts and flow
durations are measured at L4).
"""
from __future__ import annotations

import json
import os
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import httpx


def env_float(name: str, default: float) -> float:
    try:
        return float(os.environ.get(name, default))
    except ValueError:
        return default


def env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


class JsonHandler(BaseHTTPRequestHandler):
    """Base request handler: JSON bodies, CORS, SSE."""

    cors_methods = "POST, GET, OPTIONS"
    server_version = "atta-agent/1.0"

    def log_message(self, fmt, *args):  # quieter access log (stderr)
        if os.environ.get("AGENT_ACCESS_LOG", "0") == "1":
            super().log_message(fmt, *args)

    def set_cors(self):
        self.send_header("Access-Control-Allow-Origin", "*")
        self.send_header("Access-Control-Allow-Methods", self.cors_methods)
        self.send_header("Access-Control-Allow-Headers", "Content-Type")

    def send_json(self, status: int, payload) -> None:
        body = json.dumps(payload, default=str).encode("utf-8")
        self.send_response(status)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.set_cors()
        self.end_headers()
        self.wfile.write(body)

    def read_json(self):
        """Returns (data, error_response_sent)."""
        n = int(self.headers.get("Content-Length", "0") or 0)
        raw = self.rfile.read(n) if n > 0 else b""
        try:
            data = json.loads(raw.decode("utf-8")) if raw else {}
        except (json.JSONDecodeError, UnicodeDecodeError):
            self.send_json(400, {"error": "Invalid JSON"})
            return None, True
        if not isinstance(data, dict):
            self.send_json(400, {"error": "Invalid JSON"})
            return None, True
        return data, False

    def start_sse(self):
        self.send_response(200)
        self.send_header("Content-Type", "text/event-stream")
        self.send_header("Cache-Control", "no-cache")
        self.send_header("Connection", "keep-alive")
        self.set_cors()
        self.end_headers()

    def send_sse(self, event: str, data) -> None:
        msg = f"event: {event}\ndata: {json.dumps(data, default=str)}\n\n"
        self.wfile.write(msg.encode("utf-8"))
        self.wfile.flush()


def serve(handler_cls, host: str, port: int, banner: str):
    srv = ThreadingHTTPServer((host, port), handler_cls)
    srv.daemon_threads = True
    print(banner, flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        print("\n[*] Shutting down.", flush=True)
    finally:
        srv.server_close()


def start_background(handler_cls, host: str = "127.0.0.1", port: int = 0):
    """Start a ThreadingHTTPServer on a daemon thread (tests, in-process stacks).
    Returns (server, base_url)."""
    srv = ThreadingHTTPServer((host, port), handler_cls)
    srv.daemon_threads = True
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    return srv, f"http://{host}:{srv.server_address[1]}"


# ---- clients ---------------------------------------------------------------------------
_SSL_CTX = None
_SSL_LOCK = threading.Lock()


def shared_ssl_context():
    """One TLS context for every per-call client.  ``httpx.post`` builds a client per call,
    and a client built without one loads the CA bundle again: ~65 ms of GIL-holding CPU per
    call, 13 calls per agentic_parallel task - about 0.8 s of a ~5 s task on the serving
    host (bench --via http).  The per-call TCP connection is unchanged."""
    global _SSL_CTX
    if _SSL_CTX is None:
        with _SSL_LOCK:
            if _SSL_CTX is None:
                import ssl

                _SSL_CTX = ssl.create_default_context()
    return _SSL_CTX


def post_json_new_conn(url: str, payload: dict, headers: dict | None, timeout: float) -> dict:
    """One request on a fresh TCP connection (the reference's module-level httpx.post)."""
    r = httpx.post(url, json=payload, headers=headers, timeout=timeout,
                   verify=shared_ssl_context())
    r.raise_for_status()
    return r.json()


def llm_output(data: dict) -> tuple[str, dict]:
    meta = data.get("meta")
    return str(data.get("output", "")), (meta if isinstance(meta, dict) else {})
