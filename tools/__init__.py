"""Compatibility entry points for the reference's tool module paths
(``python -m tools.mcp_tool_db.server``, ``python -m tools.mcp_universe.openai_proxy``,
``python tools/mcp_servers/<name>_server.py``).  Implementations live in
``agentic_traffic_testing_amd.tools``."""
import os
import sys

_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _root not in sys.path:
    sys.path.insert(0, _root)
