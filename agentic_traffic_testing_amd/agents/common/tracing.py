"""Agent-side tracing helpers (reference agents/common/tracing.py:1-85) on utils.otel."""
from __future__ import annotations

from ...utils import otel
from ...utils.otel import SpanKind, attach, detach, extract, get_current, inject  # noqa: F401


def get_tracer(service_name: str):
    return otel.get_tracer(service_name)


def span_to_metadata(span) -> dict:
    return otel.span_metadata(span)
