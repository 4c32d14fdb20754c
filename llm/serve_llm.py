"""``python -m llm.serve_llm`` -> MI355X-native LLM backend (see
agentic_traffic_testing_amd/serving/serve_llm.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from agentic_traffic_testing_amd.serving.serve_llm import main  # noqa: E402

if __name__ == "__main__":
    main()
