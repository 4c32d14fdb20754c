"""``python -m agents.agent_b.main`` -> standalone Agent B CLI."""
import agents  # noqa: F401
from agentic_traffic_testing_amd.agents.agent_b.main import main

if __name__ == "__main__":
    main()
