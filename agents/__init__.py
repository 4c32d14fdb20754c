"""Compatibility entry points for the reference's module paths:
``python -m agents.agent_a.server`` / ``python -m agents.agent_b.server``
(infra/docker-compose.yml:78, 105).  Implementations live in
``agentic_traffic_testing_amd.agents``."""
import os
import sys

_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if _root not in sys.path:
    sys.path.insert(0, _root)
