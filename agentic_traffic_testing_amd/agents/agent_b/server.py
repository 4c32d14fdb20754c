"""Agent B worker service: ``POST /subtask`` and its ``/discuss`` alias on :8102
(reference agents/agent_b/server.py:1-232).

Request ``{subtask, scenario?, agent_b_role?, agent_b_contract?}``; headers
``X-Task-ID`` (reused as task id), ``X-Request-ID`` (forwarded to the LLM), ``x-agent-index``,
``traceparent``.  One LLM call with the prompt ``"You are Agent B.\\n<Role/Contract>\\n\\n
<subtask>"``.  Response ``{task_id, agent_id: "AgentB", output, llm_prompt, llm_response,
llm_endpoint, llm_meta, otel{agent_b, llm_backend}, llm_requests[1]}``.

Fix vs the reference: an LLM failure returns
``502 {"error": "LLM failed: ..."}`` instead of dropping the connection.
"""
from __future__ import annotations

import os
from datetime import datetime, timezone

from ..common import tracing
from ..common.http import JsonHandler, env_int, serve
from ..common.metrics_logger import MetricsLogger
from ..common.telemetry import TelemetryLogger
from . import main as client

HOST = "0.0.0.0"


def _log_prompt(label: str, prompt: str):
    if os.environ.get("LOG_LLM_REQUESTS", "").lower() not in ("1", "true", "yes", "on"):
        return
    n = max(int(os.environ.get("LLM_LOG_MAX_CHARS", "500")), 0)
    suffix = "" if len(prompt) <= n else f"... [truncated {len(prompt) - n} chars]"
    print(f"[agent-b][llm] {label} prompt_len={len(prompt)} prompt={prompt[:n]}{suffix}",
          flush=True)


def build_prompt(subtask: str, role: str | None, contract: str | None) -> str:
    ctx = "\n".join(p for p in ((f"Role: {role}" if role else ""),
                                (f"Contract: {contract}" if contract else "")) if p)
    return f"You are Agent B.\n{ctx}\n\n{subtask}" if ctx else f"You are Agent B.\n\n{subtask}"


class AgentBHandler(JsonHandler):
    cors_methods = "POST, OPTIONS"
    logger = TelemetryLogger(agent_id="AgentB")
    tracer = tracing.get_tracer("agent-b")
    metrics = MetricsLogger()

    def do_OPTIONS(self):  # noqa: N802
        self.send_response(204 if self.path in ("/subtask", "/discuss") else 404)
        self.set_cors()
        self.end_headers()

    def do_POST(self):  # noqa: N802
        if self.path not in ("/subtask", "/discuss"):
            self.send_json(404, {"error": "Not found"})
            return
        self.handle_subtask()

    def handle_subtask(self):
        hdr = self.headers
        agent_index = hdr.get("x-agent-index")
        req_id = hdr.get("X-Request-ID")
        ctx = tracing.extract({k: v for k, v in hdr.items()})
        with self.tracer.start_as_current_span("agent_b.handle_subtask", context=ctx,
                                               kind=tracing.SpanKind.SERVER) as span:
            data, err = self.read_json()
            if err:
                return
            subtask = data.get("subtask")
            scenario = data.get("scenario")
            role = data.get("agent_b_role") if isinstance(data.get("agent_b_role"), str) else None
            contract = (data.get("agent_b_contract")
                        if isinstance(data.get("agent_b_contract"), str) else None)
            if not isinstance(subtask, str) or not subtask:
                self.send_json(400, {"error": "Missing 'subtask' field"})
                return
            span.set_attribute("app.subtask", subtask)
            if scenario:
                span.set_attribute("app.scenario", scenario)
            if agent_index:
                span.set_attribute("app.agent_index", agent_index)
            if role:
                span.set_attribute("app.agent_role", role)
                span.set_attribute("app.role_service",
                                   f"{os.environ.get('OTEL_SERVICE_NAME', 'agent-b')}:{role}")
            log = self.logger
            task_id = hdr.get("X-Task-ID") or log.new_task_id()
            span.set_attribute("app.task_id", task_id)
            extra = {"agent_role": role, "agent_index": agent_index} if (role or agent_index) else None
            log.log(task_id, "subtask_received", subtask, extra=extra, scenario=scenario)
            tcid = log.new_tool_call_id()
            log.log(task_id, "llm_request", "Calling LLM server (HTTP AgentB)", tool_call_id=tcid,
                    scenario=scenario)
            prompt = build_prompt(subtask, role, contract)
            label = f"subtask_{agent_index or 'unknown'}"
            _log_prompt(label, prompt)
            llm_url = os.environ.get("LLM_SERVER_URL", client.LLM_SERVER_URL)
            with self.tracer.start_as_current_span("agent_b.call_llm",
                                                   kind=tracing.SpanKind.CLIENT) as sp_llm:
                t0 = datetime.now(timezone.utc).isoformat()
                sp_llm.set_attribute("app.request_start_time_utc", t0)
                sp_llm.set_attribute("app.llm.url", llm_url)
                headers = tracing.inject({})
                if req_id:
                    headers["X-Request-ID"] = req_id
                headers["X-Task-ID"] = task_id
                # fan-out membership for the backend's burst-aware admission
                if hdr.get("x-fanout"):
                    headers["x-fanout"] = hdr.get("x-fanout")
                    if agent_index:
                        headers["x-agent-index"] = agent_index
                try:
                    output, meta = client.call_llm(prompt, headers=headers, url=llm_url)
                except Exception as exc:
                    t1 = datetime.now(timezone.utc).isoformat()
                    self.metrics.log_call(task_id=task_id, agent_id="AgentB", call_type="sub_call",
                                          timestamp_start=t0, timestamp_end=t1, http_status=502,
                                          error=str(exc))
                    log.log(task_id, "llm_error", f"LLM call failed (HTTP AgentB): {exc}",
                            tool_call_id=tcid, scenario=scenario)
                    self.send_json(502, {"error": f"LLM failed: {exc}", "task_id": task_id})
                    return
                t1 = datetime.now(timezone.utc).isoformat()
                b_meta = tracing.span_to_metadata(sp_llm)
                self.metrics.log_call(task_id=task_id, agent_id="AgentB", call_type="sub_call",
                                      timestamp_start=t0, timestamp_end=t1, http_status=200,
                                      llm_meta=meta)
            otel_meta = {"agent_b": b_meta, "llm_backend": meta.get("otel", {})}
            llm_request = {"source": "agent_b", "label": label, "prompt": prompt,
                           "response": output, "agent_index": agent_index, "endpoint": llm_url,
                           "otel": otel_meta, "llm_meta": meta}
            log.log(task_id, "llm_response", "AgentB received LLM response (HTTP)",
                    tool_call_id=tcid, extra={"output_preview": output[:200]}, scenario=scenario)
            self.send_json(200, {
                "task_id": task_id, "agent_id": "AgentB", "output": output, "llm_prompt": prompt,
                "llm_response": output, "llm_endpoint": llm_url, "llm_meta": meta,
                "otel": otel_meta, "llm_requests": [llm_request]})


def run():
    port = env_int("AGENT_B_PORT", 8102)
    serve(AgentBHandler, HOST, port,
          f"[*] Agent B HTTP server listening on http://{HOST}:{port}/subtask and /discuss")


if __name__ == "__main__":
    run()
