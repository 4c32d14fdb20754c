"""MCP stdio client + the agents' ``MCPClientManager`` (reference agents/common/mcp_client.py).

``MCPClientManager(server_configs)`` keeps the reference's surface: ``connect_all()``
spawns each configured stdio server (``{"command", "args", "env"}``), runs the
``initialize`` handshake and caches ``tools/list``; ``call_tool(server, tool, args)``
returns the result's ``content`` list; ``list_tools(server=None)``; ``close()``; and the
module-level ``run_sync(coro)`` bridge for synchronous callers (mcp_client.py:121-137).

Own implementation (the ``mcp`` SDK is not installed): asyncio subprocess pipes carrying
newline-delimited JSON-RPC 2.0, one reader task per server resolving request futures.
Servers that fail to start are logged and skipped, as in the reference (mcp_client.py:84).
"""
from __future__ import annotations

import asyncio
import itertools
import json
import logging
import os
import sys
from dataclasses import dataclass
from typing import Any

from .server import PROTOCOL_VERSION

logger = logging.getLogger(__name__)


@dataclass
class ToolInfo:
    name: str
    description: str
    inputSchema: dict

    def __repr__(self) -> str:
        return f"Tool(name={self.name!r})"


class McpError(RuntimeError):
    pass


class StdioSession:
    """One JSON-RPC session with a stdio MCP server subprocess."""

    def __init__(self, proc: asyncio.subprocess.Process, name: str, timeout: float = 30.0):
        self.proc = proc
        self.name = name
        self.timeout = timeout
        self._ids = itertools.count(1)
        self._pending: dict[int, asyncio.Future] = {}
        self._reader = asyncio.ensure_future(self._read_loop())
        self.server_info: dict = {}

    @classmethod
    async def spawn(cls, name: str, command: str, args: list, env: dict | None = None,
                    timeout: float = 30.0) -> "StdioSession":
        full_env = dict(os.environ)
        full_env.update(env or {})
        if command in ("python", "python3"):
            command = sys.executable  # same interpreter as the caller
        proc = await asyncio.create_subprocess_exec(
            command, *map(str, args), stdin=asyncio.subprocess.PIPE,
            stdout=asyncio.subprocess.PIPE, stderr=None, env=full_env)
        return cls(proc, name, timeout)

    async def _read_loop(self):
        try:
            while True:
                line = await self.proc.stdout.readline()
                if not line:
                    break
                try:
                    msg = json.loads(line)
                except json.JSONDecodeError:
                    logger.warning("MCP %s: non-JSON line on stdout: %r", self.name, line[:200])
                    continue
                fut = self._pending.pop(msg.get("id"), None)
                if fut is not None and not fut.done():
                    fut.set_result(msg)
        finally:
            for fut in self._pending.values():
                if not fut.done():
                    fut.set_exception(McpError(f"MCP server '{self.name}' closed the pipe"))
            self._pending.clear()

    async def request(self, method: str, params: dict | None = None) -> Any:
        mid = next(self._ids)
        fut = asyncio.get_running_loop().create_future()
        self._pending[mid] = fut
        await self._send({"jsonrpc": "2.0", "id": mid, "method": method, "params": params or {}})
        msg = await asyncio.wait_for(fut, self.timeout)
        if "error" in msg:
            err = msg["error"]
            raise McpError(f"{method}: {err.get('message')} (code {err.get('code')})")
        return msg.get("result")

    async def notify(self, method: str, params: dict | None = None):
        await self._send({"jsonrpc": "2.0", "method": method, "params": params or {}})

    async def _send(self, msg: dict):
        self.proc.stdin.write((json.dumps(msg) + "\n").encode())
        await self.proc.stdin.drain()

    async def initialize(self) -> dict:
        self.server_info = await self.request("initialize", {
            "protocolVersion": PROTOCOL_VERSION, "capabilities": {},
            "clientInfo": {"name": "agentic-traffic-testbed", "version": "1.0"}})
        await self.notify("notifications/initialized")
        return self.server_info

    async def list_tools(self) -> list[ToolInfo]:
        res = await self.request("tools/list")
        return [ToolInfo(t["name"], t.get("description", ""), t.get("inputSchema", {}))
                for t in res.get("tools", [])]

    async def call_tool(self, name: str, arguments: dict) -> dict:
        return await self.request("tools/call", {"name": name, "arguments": arguments})

    async def read_resource(self, uri: str) -> dict:
        return await self.request("resources/read", {"uri": uri})

    async def close(self):
        if self.proc.returncode is None:
            try:
                self.proc.stdin.close()
            except Exception:
                pass
            try:
                await asyncio.wait_for(self.proc.wait(), 5)
            except asyncio.TimeoutError:
                self.proc.kill()
                await self.proc.wait()
        self._reader.cancel()


class MCPClientManager:
    """Manage stdio MCP server connections for an agent (reference mcp_client.py:23-118)."""

    def __init__(self, server_configs: dict[str, dict[str, Any]]):
        self._server_configs = server_configs
        self._sessions: dict[str, StdioSession] = {}
        self._tools: dict[str, list] = {}

    async def connect_all(self) -> None:
        for name, cfg in self._server_configs.items():
            if name in self._sessions:
                continue
            try:
                logger.info("Connecting to MCP server '%s' using %s %s", name,
                            cfg.get("command", "python"), cfg.get("args", []))
                s = await StdioSession.spawn(name, cfg.get("command", "python"),
                                             cfg.get("args", []), cfg.get("env", {}))
                await s.initialize()
                tools = await s.list_tools()
                self._sessions[name] = s
                self._tools[name] = tools
                logger.info("Connected to MCP server '%s' with %d tools", name, len(tools))
            except Exception as exc:
                logger.exception("Failed to connect to MCP server '%s': %s", name, exc)

    async def call_tool(self, server_name: str, tool_name: str, arguments: dict) -> Any:
        s = self._sessions.get(server_name)
        if not s:
            raise RuntimeError(f"MCP server '{server_name}' is not connected")
        res = await s.call_tool(tool_name, arguments)
        return res.get("content")

    async def read_resource(self, server_name: str, uri: str) -> Any:
        s = self._sessions.get(server_name)
        if not s:
            raise RuntimeError(f"MCP server '{server_name}' is not connected")
        return (await s.read_resource(uri)).get("contents")

    def list_tools(self, server_name: str | None = None) -> dict[str, Any]:
        if server_name is not None:
            return {server_name: self._tools.get(server_name, [])}
        return dict(self._tools)

    async def close(self) -> None:
        sessions = list(self._sessions.values())
        self._sessions.clear()
        self._tools.clear()
        for s in sessions:
            try:
                await s.close()
            except Exception:
                logger.exception("Error while closing MCP session %s", s.name)


def run_sync(coro: Any) -> Any:
    """Run an MCP coroutine from synchronous code (reference mcp_client.py:121-137)."""
    try:
        loop = asyncio.get_running_loop()
    except RuntimeError:
        loop = None
    if loop and loop.is_running():
        return asyncio.run_coroutine_threadsafe(coro, loop).result()
    return asyncio.run(coro)
