"""LLM-backend tracing init (reference llm/tracing.py:14-33): ``init_tracer(service_name)``
configures the OTLP/HTTP endpoint (default ``http://jaeger:4318/v1/traces``) and returns a
tracer; ``get_tracer(name)`` returns the process tracer.  Backed by the dependency-free
``agentic_traffic_testing_amd.utils.otel`` (the OpenTelemetry SDK is not in this image)."""
from __future__ import annotations

import os

import llm  # noqa: F401  (puts the repo root on sys.path)
from agentic_traffic_testing_amd.utils import otel

_service = "llm-backend"


def init_tracer(service_name: str = "llm-backend", endpoint: str | None = None):
    global _service
    _service = service_name
    if endpoint:
        os.environ.setdefault("OTEL_EXPORTER_OTLP_ENDPOINT", endpoint)
    return otel.get_tracer(service_name)


def get_tracer(name: str | None = None):
    return otel.get_tracer(name or _service)
