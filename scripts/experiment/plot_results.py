#!/usr/bin/env python3
"""CLI wrapper: agentic_traffic_testing_amd.experiments.plot_results."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from agentic_traffic_testing_amd.experiments.plot_results import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
