"""Coding tools MCP server (reference tools/mcp_servers/coding_server.py:18-79).

Tools: ``execute_python_code`` (fresh interpreter subprocess, 10 s limit) and
``analyze_code_complexity``; resource ``resource://code-snippets/python``.
Run: ``python -m agentic_traffic_testing_amd.tools.mcp_servers.coding_server`` (stdio).
"""
from __future__ import annotations

import subprocess
import sys

from agentic_traffic_testing_amd.tools.mcp import ToolServer

server = ToolServer("coding-tools-server")
EXEC_TIMEOUT_S = 10


@server.tool()
def execute_python_code(code: str) -> dict:
    """Run a short Python snippet in a fresh interpreter and return stdout / stderr.

    Toy-experiment sandbox only (a subprocess with a hard timeout), not for untrusted
    multi-tenant use."""
    try:
        proc = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                              timeout=EXEC_TIMEOUT_S)
    except subprocess.TimeoutExpired:
        return {"error": f"Code execution timed out after {EXEC_TIMEOUT_S} seconds.",
                "success": False}
    return {"stdout": proc.stdout, "stderr": proc.stderr, "return_code": proc.returncode,
            "success": proc.returncode == 0}


@server.tool()
def analyze_code_complexity(code: str) -> dict:
    """Basic structural statistics of a Python snippet."""
    lines = code.splitlines()
    body = [ln.lstrip() for ln in lines if ln.strip()]
    return {"lines_of_code": len(lines), "non_empty_lines": len(body),
            "function_count": sum(ln.startswith("def ") for ln in body),
            "class_count": sum(ln.startswith("class ") for ln in body)}


@server.resource("resource://code-snippets/python")
def get_python_snippets() -> str:
    """A small catalogue of common Python patterns."""
    return "\n".join([
        "Common Python Snippets:",
        "- List comprehension: [x * 2 for x in range(10)]",
        "- Dict comprehension: {k: v for k, v in items}",
        "- Error handling: try:",
        "      ...",
        "  except Exception as e:",
        "      ...",
        "",
    ])


if __name__ == "__main__":
    server.run()
