"""Reference module path ``agents.common.telemetry`` -> ``agentic_traffic_testing_amd.agents.common.telemetry`` (same module object)."""
import sys

import agents  # noqa: F401  (puts the repo root on sys.path)
import agentic_traffic_testing_amd.agents.common.telemetry as _impl

sys.modules[__name__] = _impl
