"""``python -m llm.hf_cpu_server`` -> CPU plumbing backend (BASELINE config 1).
See agentic_traffic_testing_amd/serving/cpu_server.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agentic_traffic_testing_amd.serving.cpu_server import main  # noqa: E402

if __name__ == "__main__":
    main()
