#!/usr/bin/env python3
"""CLI: run MCP-Universe benchmark domains (see agentic_traffic_testing_amd.experiments)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from agentic_traffic_testing_amd.experiments.run_mcp_universe import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
