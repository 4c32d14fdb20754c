"""mcp-tool-db: ``POST /query {query, task_id?}`` -> deterministic records on :8201.

Behaviour of reference tools/mcp_tool_db/server.py:14-91: 404 for other paths, 400 for
invalid JSON or a missing / empty ``query``, ``task_id`` defaults to ``unknown-task``,
``tool_request`` / ``tool_response`` telemetry events sharing one tool_call_id (agent id
``ToolDB``), an OTel span ``mcp_tool_db.query`` with ``app.query`` / ``app.task_id``, and
the response ``{"records": [{"id": 1, "value": "Echo of '<query>'"}]}``.

The reference serves with a single-threaded ``HTTPServer`` (server.py:78); that is kept
(one request at a time is part of its traffic shape).  It also propagates an incoming W3C
``traceparent`` so a caller's trace continues into the tool span.
"""
from __future__ import annotations

import os
from http.server import HTTPServer

from ...agents.common.http import JsonHandler
from ...agents.common.telemetry import TelemetryLogger
from ...agents.common.tracing import SpanKind, extract, get_tracer

HOST = "0.0.0.0"


def port() -> int:
    return int(os.environ.get("MCP_TOOL_DB_PORT", "8201"))


def lookup(query: str) -> dict:
    """The deterministic "database" answer."""
    return {"records": [{"id": 1, "value": f"Echo of '{query}'"}]}


class DbToolRequestHandler(JsonHandler):
    logger = TelemetryLogger(agent_id="ToolDB")
    tracer = get_tracer("mcp-tool-db")

    def do_POST(self) -> None:  # noqa: N802
        if self.path != "/query":
            self.send_json(404, {"error": "Not found"})
            return
        with self.tracer.start_as_current_span("mcp_tool_db.query", context=extract(self.headers),
                                               kind=SpanKind.SERVER) as span:
            data, sent = self.read_json()
            if sent:
                return
            query = data.get("query")
            task_id = data.get("task_id") or "unknown-task"
            if not isinstance(query, str) or not query:
                self.send_json(400, {"error": "Missing 'query' field"})
                return
            span.set_attribute("app.query", query)
            span.set_attribute("app.task_id", task_id)
            call_id = self.logger.new_tool_call_id()
            self.logger.log(task_id=task_id, event_type="tool_request",
                            message="DB tool query received", tool_call_id=call_id,
                            extra={"query_preview": query[:200]})
            result = lookup(query)
            self.logger.log(task_id=task_id, event_type="tool_response",
                            message="DB tool response sent", tool_call_id=call_id)
            self.send_json(200, result)


def make_server(host: str = HOST, listen_port: int | None = None) -> HTTPServer:
    return HTTPServer((host, port() if listen_port is None else listen_port),
                      DbToolRequestHandler)


def run() -> None:
    srv = make_server()
    print(f"[*] MCP-style DB tool listening on http://{HOST}:{srv.server_address[1]}/query",
          flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        print("\n[*] Shutting down DB tool server.")
    finally:
        srv.server_close()


if __name__ == "__main__":
    run()
