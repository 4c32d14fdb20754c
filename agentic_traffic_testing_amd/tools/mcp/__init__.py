"""Dependency-free Model Context Protocol (stdio JSON-RPC) server + client."""
from .client import MCPClientManager, StdioSession, run_sync
from .server import ToolServer

__all__ = ["MCPClientManager", "StdioSession", "ToolServer", "run_sync"]
