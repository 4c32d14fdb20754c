"""Reference path ``agents.common`` (agents/common/*.py in the reference): telemetry, metrics
logger, tracing and the MCP client manager, backed by ``agentic_traffic_testing_amd``."""
import agents  # noqa: F401
