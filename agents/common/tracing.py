"""Reference module path ``agents.common.tracing`` -> ``agentic_traffic_testing_amd.agents.common.tracing`` (same module object)."""
import sys

import agents  # noqa: F401  (puts the repo root on sys.path)
import agentic_traffic_testing_amd.agents.common.tracing as _impl

sys.modules[__name__] = _impl
