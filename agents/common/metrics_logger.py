"""Reference module path ``agents.common.metrics_logger`` -> ``agentic_traffic_testing_amd.agents.common.metrics_logger`` (same module object)."""
import sys

import agents  # noqa: F401  (puts the repo root on sys.path)
import agentic_traffic_testing_amd.agents.common.metrics_logger as _impl

sys.modules[__name__] = _impl
