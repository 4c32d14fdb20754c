"""OpenTelemetry-compatible tracing with W3C ``traceparent`` propagation.

The reference uses the OpenTelemetry SDK with an OTLP/HTTP exporter to Jaeger
(agents/common/tracing.py:16-37, llm/tracing.py:14-28) and embeds span ids in JSON
responses (``span_to_metadata``, agents/common/tracing.py:50-85).  The SDK is not part of
this image, so this module is a small self-contained implementation of the surface the
testbed uses, speaking the same wire formats (W3C trace-context headers, OTLP/HTTP JSON), so
Jaeger and any OpenTelemetry-instrumented peer interoperate with it:

* ``get_tracer(name)`` -> tracer with ``start_as_current_span(name, context=, kind=)`` and
  ``start_span``; spans carry ``set_attribute``, ``get_span_context()``, ``attributes``;
* ``inject(headers)`` / ``extract(headers)`` (W3C trace-context), ``get_current()``,
  ``attach(ctx)`` / ``detach(token)`` for carrying context into worker threads;
* a background batch exporter that POSTs OTLP/HTTP JSON to
  ``OTEL_EXPORTER_OTLP_ENDPOINT`` (default ``http://jaeger:4318/v1/traces``), best effort
  (short timeouts, bounded queue, silently drops when the collector is unreachable).
"""
from __future__ import annotations

import contextlib
import contextvars
import enum
import json
import os
import queue
import random
import threading
import time
import urllib.request

DEFAULT_ENDPOINT = "http://jaeger:4318/v1/traces"


class SpanKind(enum.IntEnum):
    INTERNAL = 1
    SERVER = 2
    CLIENT = 3
    PRODUCER = 4
    CONSUMER = 5


class SpanContext:
    __slots__ = ("trace_id", "span_id", "trace_flags", "is_remote")

    def __init__(self, trace_id: int, span_id: int, trace_flags: int = 1, is_remote=False):
        self.trace_id, self.span_id = trace_id, span_id
        self.trace_flags, self.is_remote = trace_flags, is_remote

    @property
    def is_valid(self) -> bool:
        return self.trace_id != 0 and self.span_id != 0


class Span:
    def __init__(self, name: str, ctx: SpanContext, parent: SpanContext | None,
                 kind: SpanKind, service: str, exporter):
        self.name = name
        self._ctx = ctx
        self.parent = parent
        self.kind = kind
        self.service = service
        self.attributes: dict = {}
        self.start_ns = time.time_ns()
        self.end_ns: int | None = None
        self._exporter = exporter
        self.status_error: str | None = None

    def get_span_context(self) -> SpanContext:
        return self._ctx

    def set_attribute(self, key: str, value):
        self.attributes[key] = value

    def set_attributes(self, attrs: dict):
        self.attributes.update(attrs)

    def record_exception(self, exc: BaseException):
        self.status_error = f"{type(exc).__name__}: {exc}"

    def is_recording(self) -> bool:
        return self.end_ns is None

    def end(self, end_time: int | None = None):
        if self.end_ns is None:
            self.end_ns = time.time_ns() if end_time is None else int(end_time)
            if self._exporter is not None:
                self._exporter.submit(self)


class _Ctx:
    """Immutable context object: the current span (or a remote parent)."""
    __slots__ = ("span", "remote")

    def __init__(self, span: Span | None = None, remote: SpanContext | None = None):
        self.span, self.remote = span, remote

    def span_context(self) -> SpanContext | None:
        if self.span is not None:
            return self.span.get_span_context()
        return self.remote


_current: contextvars.ContextVar[_Ctx] = contextvars.ContextVar("atta_otel_ctx", default=_Ctx())


def get_current() -> _Ctx:
    return _current.get()


def context_of(span: Span) -> _Ctx:
    """A context whose current span is ``span`` (to parent a child without entering it)."""
    return _Ctx(span=span)


def attach(ctx: _Ctx):
    return _current.set(ctx if ctx is not None else _Ctx())


def detach(token):
    with contextlib.suppress(Exception):
        _current.reset(token)


def get_current_span() -> Span | None:
    return _current.get().span


def inject(headers: dict, ctx: _Ctx | None = None) -> dict:
    sc = (ctx or _current.get()).span_context()
    if sc is not None and sc.is_valid:
        headers["traceparent"] = f"00-{sc.trace_id:032x}-{sc.span_id:016x}-{sc.trace_flags:02x}"
    return headers


def extract(headers) -> _Ctx:
    tp = None
    for k, v in dict(headers).items():
        if str(k).lower() == "traceparent":
            tp = v
            break
    if not tp:
        return _Ctx()
    try:
        ver, tid, sid, flags = tp.strip().split("-")[:4]
        sc = SpanContext(int(tid, 16), int(sid, 16), int(flags, 16), is_remote=True)
        return _Ctx(remote=sc) if sc.is_valid else _Ctx()
    except Exception:
        return _Ctx()


class _Exporter:
    """Batching OTLP/HTTP JSON exporter on a daemon thread."""

    def __init__(self, endpoint: str):
        self.endpoint = endpoint
        self.q: queue.Queue = queue.Queue(maxsize=10000)
        self.failures = 0
        self.exported = 0
        self._t = threading.Thread(target=self._run, name="otel-export", daemon=True)
        self._t.start()

    def submit(self, span: Span):
        with contextlib.suppress(queue.Full):
            self.q.put_nowait(span)

    def _run(self):
        while True:
            batch = [self.q.get()]
            deadline = time.time() + 1.0
            while len(batch) < 256 and time.time() < deadline:
                try:
                    batch.append(self.q.get(timeout=max(0.0, deadline - time.time())))
                except queue.Empty:
                    break
            if self.failures > 20:  # collector unreachable: stop trying, keep draining
                continue
            try:
                body = json.dumps(_otlp_json(batch)).encode()
                req = urllib.request.Request(self.endpoint, data=body, method="POST",
                                             headers={"Content-Type": "application/json"})
                urllib.request.urlopen(req, timeout=2).read()
                self.exported += len(batch)
                self.failures = 0
            except Exception:
                self.failures += 1


def _attr(k, v):
    if isinstance(v, bool):
        val = {"boolValue": v}
    elif isinstance(v, int):
        val = {"intValue": str(v)}
    elif isinstance(v, float):
        val = {"doubleValue": v}
    else:
        val = {"stringValue": str(v)}
    return {"key": k, "value": val}


def _otlp_json(spans: list[Span]) -> dict:
    by_service: dict[str, list] = {}
    for s in spans:
        sc = s.get_span_context()
        d = {
            "traceId": f"{sc.trace_id:032x}", "spanId": f"{sc.span_id:016x}",
            "name": s.name, "kind": int(s.kind),
            "startTimeUnixNano": str(s.start_ns), "endTimeUnixNano": str(s.end_ns or s.start_ns),
            "attributes": [_attr(k, v) for k, v in s.attributes.items()],
        }
        if s.parent is not None:
            d["parentSpanId"] = f"{s.parent.span_id:016x}"
        if s.status_error:
            d["status"] = {"code": 2, "message": s.status_error}
        by_service.setdefault(s.service, []).append(d)
    return {"resourceSpans": [
        {"resource": {"attributes": [_attr("service.name", svc)]},
         "scopeSpans": [{"scope": {"name": "agentic_traffic_testing_amd"}, "spans": sp}]}
        for svc, sp in by_service.items()]}


_exporter_singleton: _Exporter | None = None
_exp_lock = threading.Lock()


def _exporter() -> _Exporter | None:
    global _exporter_singleton
    if os.environ.get("OTEL_SDK_DISABLED", "").lower() in ("1", "true", "yes"):
        return None
    with _exp_lock:
        if _exporter_singleton is None:
            ep = os.environ.get("OTEL_EXPORTER_OTLP_ENDPOINT", DEFAULT_ENDPOINT)
            if not ep.rstrip("/").endswith("/v1/traces"):
                ep = ep.rstrip("/") + "/v1/traces"
            _exporter_singleton = _Exporter(ep)
        return _exporter_singleton


class Tracer:
    def __init__(self, service: str):
        self.service = service
        self._rand = random.Random()

    def _new_ctx(self, parent: SpanContext | None) -> SpanContext:
        tid = parent.trace_id if parent is not None and parent.is_valid else \
            self._rand.getrandbits(128) or 1
        return SpanContext(tid, self._rand.getrandbits(64) or 1, 1, False)

    def start_span(self, name: str, context: _Ctx | None = None,
                   kind: SpanKind = SpanKind.INTERNAL, attributes: dict | None = None,
                   start_time: int | None = None) -> Span:
        """``start_time``: epoch ns (OTel API), for spans recorded after the fact."""
        parent = (context if context is not None else _current.get()).span_context()
        sp = Span(name, self._new_ctx(parent), parent, kind, self.service, _exporter())
        if start_time is not None:
            sp.start_ns = int(start_time)
        if attributes:
            sp.attributes.update(attributes)
        return sp

    @contextlib.contextmanager
    def start_as_current_span(self, name: str, context: _Ctx | None = None,
                              kind: SpanKind = SpanKind.INTERNAL, attributes: dict | None = None):
        sp = self.start_span(name, context, kind, attributes)
        tok = _current.set(_Ctx(span=sp))
        try:
            yield sp
        except BaseException as e:
            sp.record_exception(e)
            raise
        finally:
            _current.reset(tok)
            sp.end()


_tracers: dict[str, Tracer] = {}


def get_tracer(name: str) -> Tracer:
    """Tracer whose service name honours OTEL_SERVICE_NAME (agents/common/tracing.py:22)."""
    service = os.environ.get("OTEL_SERVICE_NAME", name)
    t = _tracers.get(service)
    if t is None:
        t = _tracers[service] = Tracer(service)
    return t


def span_metadata(span) -> dict:
    """trace/span ids + attributes for JSON responses (agents/common/tracing.py:50-85)."""
    meta: dict = {}
    try:
        sc = span.get_span_context()
        meta["trace_id"] = f"{int(sc.trace_id):032x}"
        meta["span_id"] = f"{int(sc.span_id):016x}"
        meta["trace_flags"] = int(getattr(sc, "trace_flags", 0))
        meta["is_remote"] = bool(getattr(sc, "is_remote", False))
    except Exception:
        pass
    attrs = getattr(span, "attributes", None)
    if isinstance(attrs, dict) and attrs:
        meta["attributes"] = dict(attrs)
    return meta
