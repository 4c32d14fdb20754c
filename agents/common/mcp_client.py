"""Reference module path ``agents.common.mcp_client`` -> ``agentic_traffic_testing_amd.tools.mcp.client`` (same module object)."""
import sys

import agents  # noqa: F401  (puts the repo root on sys.path)
import agentic_traffic_testing_amd.tools.mcp.client as _impl

sys.modules[__name__] = _impl
