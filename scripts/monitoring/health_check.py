#!/usr/bin/env python3
"""CLI: testbed health check (exit 0 = all critical checks passed)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from agentic_traffic_testing_amd.observability.health_check import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
