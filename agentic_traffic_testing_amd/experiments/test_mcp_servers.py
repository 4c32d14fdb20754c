"""MCP smoke run (reference scripts/experiment/test_mcp_servers.py:1-73): start the coding,
finance and maps stdio servers, list their tools and call one tool on each."""
from __future__ import annotations

import asyncio
import json
import sys

from ..tools.mcp import MCPClientManager

SERVERS = ("coding", "finance", "maps")


def server_configs() -> dict:
    return {name: {"command": sys.executable,
                   "args": ["-m", f"agentic_traffic_testing_amd.tools.mcp_servers.{name}_server"]}
            for name in SERVERS}


CALLS = (
    ("coding", "execute_python_code", {"code": "print('Hello from MCP coding server'); x = 2 + 2"}),
    ("finance", "get_stock_price", {"symbol": "AAPL"}),
    ("maps", "calculate_distance", {"location1": "New York", "location2": "London"}),
)


async def smoke(verbose: bool = True) -> dict:
    client = MCPClientManager(server_configs())
    await client.connect_all()
    out = {"tools": {k: [t.name for t in v] for k, v in client.list_tools().items()}}
    try:
        if verbose:
            print("=== Available MCP tools ===")
            print(client.list_tools())
        for server, tool, args in CALLS:
            res = await client.call_tool(server, tool, args)
            out[f"{server}.{tool}"] = json.loads(res[0]["text"])
            if verbose:
                print(f"\n=== {server}: {tool} ===")
                print(res)
    finally:
        await client.close()
    return out


def main() -> int:
    asyncio.run(smoke())
    return 0


if __name__ == "__main__":
    sys.exit(main())
