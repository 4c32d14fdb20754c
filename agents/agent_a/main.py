"""``python -m agents.agent_a.main`` -> standalone Agent A CLI."""
import agents  # noqa: F401
from agentic_traffic_testing_amd.agents.agent_a.main import main

if __name__ == "__main__":
    main()
