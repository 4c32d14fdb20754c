"""Reference module path ``agents.agent_a.orchestrator`` -> ``agentic_traffic_testing_amd.agents.agent_a.orchestrator`` (same module object)."""
import sys

import agents  # noqa: F401  (puts the repo root on sys.path)
import agentic_traffic_testing_amd.agents.agent_a.orchestrator as _impl

sys.modules[__name__] = _impl
