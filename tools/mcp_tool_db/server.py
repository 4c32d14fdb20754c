"""``python -m tools.mcp_tool_db.server`` -> agentic_traffic_testing_amd.tools.mcp_tool_db."""
import tools  # noqa: F401
from agentic_traffic_testing_amd.tools.mcp_tool_db.server import run

if __name__ == "__main__":
    run()
