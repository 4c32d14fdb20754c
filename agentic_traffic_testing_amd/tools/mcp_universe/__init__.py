"""MCP-Universe integration (reference tools/mcp_universe/__init__.py:1-51).

The benchmark framework itself is not vendored: point ``MCP_UNIVERSE_DIR`` at a checkout.
This package provides the OpenAI-compatible proxy that lets MCP-Universe's OpenAI client
talk to the local ``/chat`` backend (``openai_proxy``); the runner lives in
``agentic_traffic_testing_amd.experiments.run_mcp_universe``.
"""
from __future__ import annotations

__all__ = ["DEFAULT_OPENAI_PROXY_HOST", "DEFAULT_OPENAI_PROXY_PORT"]

DEFAULT_OPENAI_PROXY_HOST = "0.0.0.0"
DEFAULT_OPENAI_PROXY_PORT = 8110
