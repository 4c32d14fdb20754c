#!/usr/bin/env python3
"""CLI: MCP smoke test of the coding / finance / maps stdio servers."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from agentic_traffic_testing_amd.experiments.test_mcp_servers import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
