"""Minimal Model Context Protocol server over stdio (JSON-RPC 2.0, newline-delimited).

The reference's demo tool servers are written against ``fastmcp.FastMCP``
(tools/mcp_servers/coding_server.py:18-63, finance_server.py:17-98, maps_server.py:16-104)
and driven by the ``mcp`` SDK client (agents/common/mcp_client.py:16-118).  Neither package
exists in this image, so the testbed carries its own small, dependency-free implementation
of the subset those files use:

* ``ToolServer.tool()`` / ``ToolServer.resource(uri)`` decorators (same shape as FastMCP);
* JSON-RPC methods ``initialize``, ``notifications/initialized``, ``ping``, ``tools/list``
  (input schemas derived from type hints), ``tools/call`` (text content + structured
  result, ``isError`` on tool exceptions), ``resources/list``, ``resources/read``;
* stdio transport: one JSON message per line on stdin / stdout, logs on stderr.

The wire format follows the public MCP stdio transport, so a real MCP client can talk to
these servers and ``client.MCPClientManager`` can talk to real MCP servers.
"""
from __future__ import annotations

import inspect
import json
import sys
import traceback
import typing
from dataclasses import dataclass, field

PROTOCOL_VERSION = "2024-11-05"

_JSON_TYPES = {str: "string", int: "integer", float: "number", bool: "boolean",
               dict: "object", list: "array"}


def _schema_for(tp) -> dict:
    origin = typing.get_origin(tp)
    if origin in (dict, typing.Dict):
        args = typing.get_args(tp)
        sch = {"type": "object"}
        if len(args) == 2:
            sch["additionalProperties"] = _schema_for(args[1])
        return sch
    if origin in (list, typing.List):
        args = typing.get_args(tp)
        return {"type": "array", "items": _schema_for(args[0]) if args else {}}
    if origin is typing.Union:
        opts = [a for a in typing.get_args(tp) if a is not type(None)]
        return _schema_for(opts[0]) if len(opts) == 1 else {}
    return {"type": _JSON_TYPES[tp]} if tp in _JSON_TYPES else {}


def input_schema(fn) -> dict:
    sig = inspect.signature(fn)
    hints = typing.get_type_hints(fn)
    props, required = {}, []
    for name, p in sig.parameters.items():
        props[name] = _schema_for(hints.get(name, str))
        if p.default is inspect.Parameter.empty:
            required.append(name)
        else:
            props[name]["default"] = p.default
    return {"type": "object", "properties": props, "required": required}


@dataclass
class _Tool:
    name: str
    fn: typing.Callable
    description: str
    schema: dict


@dataclass
class _Resource:
    uri: str
    fn: typing.Callable
    name: str
    description: str
    mime: str = "text/plain"


@dataclass
class ToolServer:
    name: str
    version: str = "1.0.0"
    tools: dict = field(default_factory=dict)
    resources: dict = field(default_factory=dict)

    # -- registration (FastMCP-style decorators) -----------------------------------------
    def tool(self, name: str | None = None, description: str | None = None):
        def deco(fn):
            doc = inspect.cleandoc(fn.__doc__ or "")
            self.tools[name or fn.__name__] = _Tool(name or fn.__name__, fn,
                                                    description or doc, input_schema(fn))
            return fn
        return deco

    def resource(self, uri: str, name: str | None = None, mime_type: str | None = None):
        def deco(fn):
            ret = typing.get_type_hints(fn).get("return")
            mime = mime_type or ("text/plain" if ret is str else "application/json")
            self.resources[uri] = _Resource(uri, fn, name or fn.__name__,
                                            inspect.cleandoc(fn.__doc__ or ""), mime)
            return fn
        return deco

    # -- JSON-RPC dispatch ---------------------------------------------------------------
    def handle(self, msg: dict) -> dict | None:
        """Process one JSON-RPC message; returns the response (None for notifications)."""
        mid = msg.get("id")
        method = msg.get("method")
        params = msg.get("params") or {}
        if method is None:
            return None  # a response to something we never send
        try:
            result = self._dispatch(method, params)
        except _RpcError as e:
            return None if mid is None else {"jsonrpc": "2.0", "id": mid,
                                             "error": {"code": e.code, "message": str(e)}}
        if mid is None:
            return None
        return {"jsonrpc": "2.0", "id": mid, "result": result}

    def _dispatch(self, method: str, params: dict):
        if method == "initialize":
            return {"protocolVersion": params.get("protocolVersion", PROTOCOL_VERSION),
                    "capabilities": {"tools": {"listChanged": False},
                                     "resources": {"listChanged": False, "subscribe": False}},
                    "serverInfo": {"name": self.name, "version": self.version}}
        if method.startswith("notifications/"):
            return {}
        if method == "ping":
            return {}
        if method == "tools/list":
            return {"tools": [{"name": t.name, "description": t.description,
                               "inputSchema": t.schema} for t in self.tools.values()]}
        if method == "tools/call":
            return self.call_tool(params.get("name"), params.get("arguments") or {})
        if method == "resources/list":
            return {"resources": [{"uri": r.uri, "name": r.name, "description": r.description,
                                   "mimeType": r.mime} for r in self.resources.values()]}
        if method == "resources/read":
            return self.read_resource(params.get("uri"))
        raise _RpcError(-32601, f"Method not found: {method}")

    def call_tool(self, name: str, arguments: dict) -> dict:
        t = self.tools.get(name)
        if t is None:
            raise _RpcError(-32602, f"Unknown tool: {name}")
        try:
            out = t.fn(**arguments)
        except TypeError as e:
            return {"content": [{"type": "text", "text": f"Invalid arguments: {e}"}],
                    "isError": True}
        except Exception as e:  # tool failure is a result, not a protocol error
            return {"content": [{"type": "text", "text": f"{type(e).__name__}: {e}"}],
                    "isError": True}
        text = out if isinstance(out, str) else json.dumps(out, default=str)
        res = {"content": [{"type": "text", "text": text}], "isError": False}
        if isinstance(out, dict):
            res["structuredContent"] = out
        return res

    def read_resource(self, uri: str) -> dict:
        r = self.resources.get(uri)
        if r is None:
            raise _RpcError(-32002, f"Resource not found: {uri}")
        out = r.fn()
        text = out if isinstance(out, str) else json.dumps(out, default=str)
        return {"contents": [{"uri": uri, "mimeType": r.mime, "text": text}]}

    # -- stdio transport -----------------------------------------------------------------
    def run(self, stdin=None, stdout=None) -> None:
        stdin = stdin or sys.stdin
        stdout = stdout or sys.stdout
        for line in stdin:
            line = line.strip()
            if not line:
                continue
            try:
                msg = json.loads(line)
            except json.JSONDecodeError:
                resp = {"jsonrpc": "2.0", "id": None,
                        "error": {"code": -32700, "message": "Parse error"}}
            else:
                try:
                    resp = self.handle(msg) if isinstance(msg, dict) else None
                except Exception:  # keep serving; report on stderr
                    traceback.print_exc(file=sys.stderr)
                    resp = {"jsonrpc": "2.0", "id": msg.get("id"),
                            "error": {"code": -32603, "message": "Internal error"}}
            if resp is not None:
                stdout.write(json.dumps(resp) + "\n")
                stdout.flush()


class _RpcError(Exception):
    def __init__(self, code: int, message: str):
        super().__init__(message)
        self.code = code
