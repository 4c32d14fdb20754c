"""``python -m agents.agent_b.server`` -> agentic_traffic_testing_amd.agents.agent_b.server."""
import agents  # noqa: F401
from agentic_traffic_testing_amd.agents.agent_b.server import run

if __name__ == "__main__":
    run()
