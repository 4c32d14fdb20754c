"""``python tools/mcp_servers/coding_server.py`` -> stdio MCP server
(agentic_traffic_testing_amd.tools.mcp_servers.coding_server)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from agentic_traffic_testing_amd.tools.mcp_servers.coding_server import server  # noqa: E402

if __name__ == "__main__":
    server.run()
