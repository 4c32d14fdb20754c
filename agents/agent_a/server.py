"""``python -m agents.agent_a.server`` -> agentic_traffic_testing_amd.agents.agent_a.server."""
import agents  # noqa: F401  (puts the repo root on sys.path)
from agentic_traffic_testing_amd.agents.agent_a.server import run

if __name__ == "__main__":
    run()
