#!/usr/bin/env python3
"""CLI: Docker id -> name mapping exporter on :9101."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from agentic_traffic_testing_amd.observability.docker_mapping_exporter import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
