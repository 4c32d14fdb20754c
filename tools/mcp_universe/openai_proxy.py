"""``python -m tools.mcp_universe.openai_proxy`` -> the OpenAI-compatible proxy."""
import tools  # noqa: F401
from agentic_traffic_testing_amd.tools.mcp_universe.openai_proxy import main

if __name__ == "__main__":
    main()
