"""Agent A orchestrator service on :8101 (reference agents/agent_a/server.py:1-925).

Endpoints
* ``POST /task`` ``{task, scenario?, agent_a_role?, agent_a_contract?, agent_b_role?,
  agent_b_contract?, agent_count?, agent_b_workers?[{endpoint?, role?, contract?}],
  max_agent_turns?}``; scenarios
    - ``agentic_simple``    : one LLM call with the raw task;
    - ``agentic_multi_hop`` : per turn (<= MAX_AGENT_B_TURNS) one Agent B call + one Agent A
                              progress check, then a final call (2*turns + 1 LLM calls);
    - ``agentic_parallel``  : planning call -> N (<= MAX_PARALLEL_WORKERS) concurrent Agent B
                              calls (thread pool) -> planner/critic final call.
  Response: task_id, agent_id, scenario, task_query, task_start, task_end, total_llm_calls,
  total_prompt_tokens, total_completion_tokens, total_tokens, total_latency_ms,
  llm_latency_ms, total_agent_hops, cost_estimate_usd, output, agent_b_output,
  agent_b_outputs, agent_a_progress_notes, llm_requests.
* ``POST /agentverse`` ``{task, max_iterations? (1..5, default 3), success_threshold?
  (0..100, default 70), stream?}`` -> AgentVerse result JSON or an SSE stream ending in
  ``complete`` (or ``error``); runs are persisted to ``logs/agentverse/<task_id>.json``.
* ``GET /agentverse/<task_id>`` and ``GET /agentverse?task_id=|taskId=`` -> persisted run.
* ``OPTIONS`` for CORS.

Per-call connection behaviour matches the reference: /task helper calls open a new TCP
connection each (main.py), the AgentVerse orchestrator uses one keep-alive client.
"""
from __future__ import annotations

import json
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor, as_completed
from datetime import datetime, timezone
from urllib.parse import parse_qs, urlparse

import httpx

from ..common import tracing
from ..common.http import JsonHandler, env_float, env_int, serve
from ..common.metrics_logger import MetricsLogger
from ..common.telemetry import TelemetryLogger
from . import main as client
from .orchestrator import AgentVerseOrchestrator

HOST = "0.0.0.0"
CONTEXT_PREVIEW_LEN = 300


def _now() -> str:
    return datetime.now(timezone.utc).isoformat()


def _clean(v) -> str | None:
    return v.strip() if isinstance(v, str) and v.strip() else None


def normalize_workers(count, payloads, fallback_urls, cap: int | None = None) -> list[dict]:
    """N worker slots (default: one per configured Agent B URL, capped at
    MAX_PARALLEL_WORKERS); explicit per-worker endpoint/role/contract override defaults."""
    cap = cap if cap is not None else env_int("MAX_PARALLEL_WORKERS", 5)
    urls = [u for u in fallback_urls if u] or ["http://agent-b:8102/subtask"]
    n = count if isinstance(count, int) and count > 0 else len(urls)
    n = min(n, cap)
    items = payloads if isinstance(payloads, list) else []
    out = []
    for i in range(n):
        p = items[i] if i < len(items) and isinstance(items[i], dict) else {}
        out.append({"endpoint": _clean(p.get("endpoint")) or urls[i % len(urls)],
                    "role": _clean(p.get("role")), "contract": _clean(p.get("contract"))})
    return out


def parse_subtasks(raw: str, n: int, task: str) -> list[str]:
    """JSON array (or {"subtasks": [...]}) of subtasks, padded with generic
    "Subtask i: <task>" entries - the fallback that keeps the fan-out shape even when the
    planner's reply does not parse (e.g. random-init weights)."""
    try:
        parsed = json.loads(raw)
    except (json.JSONDecodeError, TypeError, ValueError):
        parsed = None
    items = parsed.get("subtasks") if isinstance(parsed, dict) else parsed
    subs = [str(s).strip() for s in items if str(s).strip()] if isinstance(items, list) else []
    subs += [f"Subtask {i + 1}: {task}" for i in range(len(subs), n)]
    return subs[:n]


def _log_prompt(label: str, prompt: str):
    if os.environ.get("LOG_LLM_REQUESTS", "").lower() not in ("1", "true", "yes", "on"):
        return
    n = max(env_int("LLM_LOG_MAX_CHARS", 500), 0)
    suffix = "" if len(prompt) <= n else f"... [truncated {len(prompt) - n} chars]"
    print(f"[agent-a][llm] {label} prompt_len={len(prompt)} prompt={prompt[:n]}{suffix}",
          flush=True)


class TaskRun:
    """State of one /task request."""

    def __init__(self, handler: "AgentAHandler", task: str, scenario, roles: dict):
        self.h = handler
        self.task = task
        self.scenario = scenario
        self.log = handler.logger
        self.task_id = self.log.new_task_id()
        self.start = _now()
        self.llm_requests: list[dict] = []
        self.b_outputs: list = []
        self.notes: list[str] = []
        r = roles
        ctx = [f"Role: {r['a_role']}" if r["a_role"] else "",
               f"Contract: {r['a_contract']}" if r["a_contract"] else ""]
        ctx = "\n".join(c for c in ctx if c)
        self.role_block = f"{ctx}\n" if ctx else ""
        self.roles = r

    def ev(self, event: str, msg: str, **kw):
        self.log.log(self.task_id, event, msg, scenario=self.scenario, **kw)

    def llm(self, label: str, prompt: str, span_name: str, call_type: str, **entry_extra):
        """One Agent A -> LLM call on a fresh connection, logged + recorded."""
        with self.h.tracer.start_as_current_span(span_name, kind=tracing.SpanKind.CLIENT) as sp:
            sp.set_attribute("app.llm.url", client.llm_url())
            for k, v in entry_extra.items():
                if k == "turn":
                    sp.set_attribute("app.turn", v)
            headers = tracing.inject({})
            headers["X-Task-ID"] = self.task_id
            _log_prompt(label, prompt)
            entry = {"source": "agent_a", "label": label, "prompt": prompt,
                     "endpoint": client.llm_url(), **entry_extra}
            self.llm_requests.append(entry)
            t0 = _now()
            out, meta = client.call_llm(prompt, headers=headers)
            entry["response"] = out
            entry["llm_meta"] = meta
            self.h.metrics.log_call(task_id=self.task_id, agent_id="AgentA", call_type=call_type,
                                    timestamp_start=t0, timestamp_end=_now(), http_status=200,
                                    llm_meta=meta)
            return out

    def aggregates(self) -> dict:
        end = _now()
        pt = ct = tt = lat = hops = 0
        for r in self.llm_requests:
            m = r.get("llm_meta") or {}
            pt += m.get("prompt_tokens") or 0
            ct += m.get("completion_tokens") or 0
            tt += m.get("total_tokens") or 0
            lat += m.get("latency_ms") or 0
            hops += r.get("source") == "agent_b"
        try:
            total_ms = int((datetime.fromisoformat(end) -
                            datetime.fromisoformat(self.start)).total_seconds() * 1000)
        except ValueError:
            total_ms = None
        ri = env_float("COST_PER_INPUT_TOKEN_USD", 0.0)
        ro = env_float("COST_PER_OUTPUT_TOKEN_USD", 0.0)
        cost = round(pt * ri + ct * ro, 8) if (ri or ro) else None
        return {"task_end": end, "total_llm_calls": len(self.llm_requests),
                "total_prompt_tokens": pt, "total_completion_tokens": ct, "total_tokens": tt,
                "total_latency_ms": total_ms, "llm_latency_ms": lat, "total_agent_hops": hops,
                "cost_estimate_usd": cost}


class AgentAHandler(JsonHandler):
    logger = TelemetryLogger(agent_id="AgentA")
    tracer = tracing.get_tracer("agent-a")
    metrics = MetricsLogger()

    # ---- routing -------------------------------------------------------------------------
    def do_OPTIONS(self):  # noqa: N802
        ok = self.path == "/task" or self.path.startswith("/agentverse")
        self.send_response(204 if ok else 404)
        self.set_cors()
        self.end_headers()

    def do_GET(self):  # noqa: N802
        u = urlparse(self.path)
        if not u.path.startswith("/agentverse"):
            if u.path in ("/health", "/ready", "/live"):
                self.send_json(200, {"status": "ok"})
                return
            self.send_json(404, {"error": "Not found"})
            return
        tid = u.path[len("/agentverse/"):].strip("/") if u.path.startswith("/agentverse/") else ""
        if not tid:
            q = parse_qs(u.query or "")
            vals = q.get("task_id") or q.get("taskId")
            tid = vals[0] if vals else ""
        if not tid:
            self.send_json(400, {"error": "Missing task_id"})
            return
        self.get_agentverse_run(tid)

    def do_POST(self):  # noqa: N802
        if self.path == "/agentverse":
            self.handle_agentverse()
        elif self.path == "/task":
            self.handle_task()
        else:
            self.send_json(404, {"error": "Not found"})

    # ---- AgentVerse ----------------------------------------------------------------------
    @staticmethod
    def runs_dir() -> str:
        return os.path.join(os.environ.get("AGENTVERSE_LOG_DIR", "logs"), "agentverse")

    def get_agentverse_run(self, task_id: str):
        task_id = task_id.strip()
        if not task_id or not all(c.isalnum() or c in "-_" for c in task_id):
            self.send_json(400, {"error": "Invalid task_id"})
            return
        path = os.path.join(self.runs_dir(), f"{task_id}.json")
        if not os.path.exists(path):
            self.send_json(404, {"error": "Task not found", "task_id": task_id})
            return
        try:
            with open(path, encoding="utf-8") as f:
                rec = json.load(f)
        except Exception as exc:
            self.send_json(500, {"error": f"Failed to load task: {exc}"})
            return
        self.send_json(200, rec)

    def persist_run(self, task_id, task, max_it, thr, result):
        try:
            d = self.runs_dir()
            os.makedirs(d, exist_ok=True)
            rec = {"task_id": task_id, "task": task, "max_iterations": max_it,
                   "success_threshold": thr, "created_at_utc": _now(), "result": result}
            with open(os.path.join(d, f"{task_id}.json"), "w", encoding="utf-8") as f:
                json.dump(rec, f, ensure_ascii=False, indent=2, default=str)
        except Exception as exc:
            print(f"[agent-a][agentverse] Failed to persist run {task_id}: {exc}", flush=True)

    def handle_agentverse(self):
        with self.tracer.start_as_current_span("agent_a.agentverse_workflow") as span:
            data, err = self.read_json()
            if err:
                return
            task = data.get("task")
            if not isinstance(task, str) or not task:
                self.send_json(400, {"error": "Missing 'task' field"})
                return
            mi = data.get("max_iterations", 3)
            mi = min(mi if isinstance(mi, int) and not isinstance(mi, bool) and mi >= 1 else 3, 5)
            thr = data.get("success_threshold", 70)
            thr = min(100, max(0, int(thr))) if isinstance(thr, (int, float)) and \
                not isinstance(thr, bool) else 70
            stream = bool(data.get("stream", False))
            for k, v in (("app.task", task), ("app.max_iterations", mi),
                         ("app.success_threshold", thr), ("app.stream", stream)):
                span.set_attribute(k, v)
            log = TelemetryLogger(agent_id="AgentA-Orchestrator", scenario="agentic_verse")
            task_id = log.new_task_id()
            span.set_attribute("app.task_id", task_id)
            log.log(task_id, "agentverse_request_received",
                    f"Received AgentVerse request: {task[:100]}...",
                    extra={"max_iterations": mi, "stream": stream})
            try:
                if stream:
                    self.start_sse()
                    lock = threading.Lock()

                    def cb(ev):
                        with lock:  # worker threads emit concurrently
                            try:
                                self.send_sse(ev["event"], ev["data"])
                            except (BrokenPipeError, ConnectionResetError):
                                pass

                    orch = AgentVerseOrchestrator(logger=log, tracer=self.tracer,
                                                  progress_callback=cb)
                    result = orch.run_workflow(task, task_id, mi, thr)
                    self.persist_run(task_id, task, mi, thr, result)
                    with lock:
                        self.send_sse("complete", result)
                    # the SSE headers asked for keep-alive; end the stream once complete
                    self.close_connection = True
                else:
                    orch = AgentVerseOrchestrator(logger=log, tracer=self.tracer)
                    result = orch.run_workflow(task, task_id, mi, thr)
                    self.persist_run(task_id, task, mi, thr, result)
                    self.send_json(200, result)
            except Exception as exc:
                log.log(task_id, "agentverse_error", f"AgentVerse workflow failed: {exc}")
                if stream:
                    self.send_sse("error", {"error": str(exc)})
                    self.close_connection = True
                else:
                    self.send_json(502, {"error": f"AgentVerse workflow failed: {exc}"})

    # ---- /task ---------------------------------------------------------------------------
    def handle_task(self):
        with self.tracer.start_as_current_span("agent_a.handle_task") as span:
            data, err = self.read_json()
            if err:
                return
            task = data.get("task")
            if not isinstance(task, str) or not task:
                self.send_json(400, {"error": "Missing 'task' field"})
                return
            scenario = data.get("scenario")
            s = lambda k: data.get(k) if isinstance(data.get(k), str) else None  # noqa: E731
            roles = {"a_role": s("agent_a_role"), "a_contract": s("agent_a_contract"),
                     "b_role": s("agent_b_role"), "b_contract": s("agent_b_contract")}
            span.set_attribute("app.task", task)
            if scenario:
                span.set_attribute("app.scenario", scenario)
            if roles["a_role"]:
                span.set_attribute("app.agent_role", roles["a_role"])
                span.set_attribute("app.role_service",
                                   f"{os.environ.get('OTEL_SERVICE_NAME', 'agent-a')}:{roles['a_role']}")
            run = TaskRun(self, task, scenario, roles)
            span.set_attribute("app.task_id", run.task_id)
            run.ev("task_received", task,
                   extra={"agent_role": roles["a_role"]} if roles["a_role"] else None)
            max_turns = env_int("MAX_AGENT_B_TURNS", 3)
            req_turns = data.get("max_agent_turns")
            if isinstance(req_turns, int) and req_turns > 0:
                max_turns = min(req_turns, max_turns)

            b_output = None
            if scenario == "agentic_parallel":
                final_prompt, b_output = self.scenario_parallel(run, data)
            elif scenario == "agentic_multi_hop":
                r = self.scenario_multi_hop(run, max_turns)
                if r is None:
                    return  # 502 already sent
                final_prompt, b_output = r
            else:
                final_prompt = task  # agentic_simple (roles ignored, as in the reference)

            tcid = run.log.new_tool_call_id()
            run.ev("llm_request", "Calling LLM server (HTTP AgentA)", tool_call_id=tcid)
            try:
                output = run.llm("final", final_prompt, "agent_a.call_llm", "root")
            except Exception as exc:
                run.ev("llm_error", f"LLM call failed (HTTP AgentA): {exc}", tool_call_id=tcid)
                self.send_json(502, {"error": f"LLM failed: {exc}"})
                return
            run.ev("llm_response", "Received LLM response (HTTP AgentA)", tool_call_id=tcid,
                   extra={"output_preview": output[:200]})
            resp = {"task_id": run.task_id, "agent_id": "AgentA", "scenario": scenario,
                    "task_query": task, "task_start": run.start}
            resp.update(run.aggregates())
            resp.update({"output": output, "agent_b_output": b_output,
                         "agent_b_outputs": run.b_outputs, "agent_a_progress_notes": run.notes,
                         "llm_requests": run.llm_requests})
            self.send_json(200, resp)

    def scenario_parallel(self, run: TaskRun, data: dict):
        task, r = run.task, run.roles
        workers = normalize_workers(data.get("agent_count"), data.get("agent_b_workers"),
                                    client.agent_b_urls())
        run.ev("agent_a_parallel_setup", "Planning parallel subtasks",
               extra={"worker_count": len(workers)})
        plan_prompt = ("You are Agent A, acting as the planner. Break the user task into "
                       f"{len(workers)} concrete, independent subtasks. Return ONLY valid JSON "
                       'as an array of strings, e.g. ["subtask 1", "subtask 2"].\n\n'
                       f"{run.role_block}User task:\n{task}")
        try:
            raw = run.llm("planning", plan_prompt, "agent_a.plan_subtasks", "sub_call")
        except Exception as exc:
            run.ev("agent_a_planning_error", f"Planning failed: {exc}")
            raw = "[]"
        subtasks = parse_subtasks(raw, len(workers), task)
        run.ev("agent_a_planning_complete", "Subtasks planned", extra={"subtasks": subtasks})
        ctx = tracing.get_current()
        b_timeout = env_float("AGENT_B_TIMEOUT_SECONDS", 120.0)

        def call_worker(idx, w, sub):
            tok = tracing.attach(ctx)
            role = w["role"] or r["b_role"]
            try:
                with self.tracer.start_as_current_span("agent_a.call_agent_b_parallel",
                                                       kind=tracing.SpanKind.CLIENT) as sp:
                    sp.set_attribute("app.agent_b.url", w["endpoint"] or "")
                    sp.set_attribute("app.agent_index", idx)
                    if role:
                        sp.set_attribute("app.agent_role", role)
                    headers = tracing.inject({"x-agent-index": str(idx)})
                    headers["X-Task-ID"] = run.task_id
                    # x-fanout: additive header for the backend's burst-aware admission
                    # (docs/agents.md); AGENT_FANOUT_HEADER=0 keeps the L7 bytes reference-exact
                    if os.environ.get("AGENT_FANOUT_HEADER", "1") != "0":
                        headers["x-fanout"] = str(len(workers))
                    # AGENT_FANOUT_STAGGER_MS: worker i's call leaves i * ms late - an L7
                    # arrival-skew knob for burst experiments (netem skews at L3)
                    stagger = env_float("AGENT_FANOUT_STAGGER_MS", 0.0) / 1000.0
                    if stagger > 0:
                        time.sleep(stagger * (idx - 1))
                    return client.call_agent_b(sub, scenario=run.scenario, headers=headers,
                                               agent_b_role=role,
                                               agent_b_contract=w["contract"] or r["b_contract"],
                                               agent_b_url_override=w["endpoint"])
            finally:
                tracing.detach(tok)

        with ThreadPoolExecutor(max_workers=max(1, len(workers))) as pool:
            fut = {}
            for idx, (w, sub) in enumerate(zip(workers, subtasks), start=1):
                tcid = run.log.new_tool_call_id()
                run.ev("agent_b_request", f"Calling worker {idx} for parallel subtask",
                       tool_call_id=tcid,
                       extra={"url": w["endpoint"], "agent_index": idx,
                              "agent_role": w["role"] or r["b_role"],
                              "subtask_preview": sub[:CONTEXT_PREVIEW_LEN]})
                fut[pool.submit(call_worker, idx, w, sub)] = (idx, w, sub)
            for f in as_completed(fut):
                idx, w, sub = fut[f]
                role = w["role"] or r["b_role"]
                try:
                    resp = f.result()
                    out = str(resp.get("output", ""))
                    ep = resp.get("llm_endpoint") or client.llm_url()
                    run.b_outputs.append({"agent_index": idx, "endpoint": w["endpoint"],
                                          "subtask": sub, "output": out,
                                          "llm_prompt": resp.get("llm_prompt"),
                                          "llm_response": resp.get("llm_response"),
                                          "llm_endpoint": ep})
                    if resp.get("llm_prompt"):
                        run.llm_requests.append({
                            "source": "agent_b", "label": "subtask",
                            "prompt": resp.get("llm_prompt"), "response": resp.get("llm_response"),
                            "agent_index": idx, "endpoint": ep,
                            "llm_meta": resp.get("llm_meta") or {}})
                    run.ev("agent_b_response", f"Worker {idx} completed",
                           extra={"output_preview": out[:200], "agent_role": role})
                except Exception as exc:
                    if isinstance(exc, httpx.TimeoutException) or "timed out" in str(exc).lower():
                        lbl = (f"{int(b_timeout)}s" if float(b_timeout).is_integer()
                               else f"{b_timeout:.1f}s")
                        text = f"Worker timed out after {lbl}"
                    else:
                        text = f"Worker failed: {exc}"
                    run.ev("agent_b_error", f"Worker {idx} failed: {exc}",
                           extra={"agent_role": role})
                    run.b_outputs.append({"agent_index": idx, "endpoint": w["endpoint"],
                                          "subtask": sub, "output": text})
        lines = []
        for idx, w in enumerate(workers, start=1):
            item = next((o for o in run.b_outputs if o["agent_index"] == idx), None)
            sub = item["subtask"] if item else (subtasks[idx - 1] if idx - 1 < len(subtasks) else "")
            lines.append(f"Worker {idx} ({w['endpoint']}):\nSubtask: {sub}\n"
                         f"{item['output'] if item else ''}")
        summary = "\n\n".join(lines)
        final = ("You are Agent A acting as planner/critic. Review the worker reports, note "
                 "inconsistencies or gaps, then produce the best final response to the user.\n\n"
                 f"{run.role_block}User task:\n{task}\n\nWorker reports:\n{summary}")
        return final, summary

    def scenario_multi_hop(self, run: TaskRun, max_turns: int):
        task, r = run.task, run.roles
        context = ""
        outputs = []
        for turn in range(1, max_turns + 1):
            sub = (f"[Turn {turn}] Help solve the user task. Provide concrete steps or "
                   f"intermediate results.\nUser task:\n{task}\n\nContext so far:\n"
                   f"{context or '(none yet)'}")
            tcid = run.log.new_tool_call_id()
            run.ev("agent_b_request", f"Calling Agent B (multi-hop, turn {turn})", tool_call_id=tcid,
                   extra={"url": client.agent_b_url(), "turn": turn,
                          "context_preview": context[:CONTEXT_PREVIEW_LEN]})
            try:
                with self.tracer.start_as_current_span("agent_a.call_agent_b",
                                                       kind=tracing.SpanKind.CLIENT) as sp:
                    sp.set_attribute("app.agent_b.url", client.agent_b_url())
                    sp.set_attribute("app.agent_b.scenario", run.scenario or "")
                    sp.set_attribute("app.turn", turn)
                    headers = tracing.inject({})
                    headers["X-Task-ID"] = run.task_id
                    resp = client.call_agent_b(sub, scenario=run.scenario, headers=headers,
                                               agent_b_role=r["b_role"],
                                               agent_b_contract=r["b_contract"])
            except Exception as exc:
                run.ev("agent_b_error", f"Agent B call failed (turn {turn}): {exc}",
                       tool_call_id=tcid)
                self.send_json(502, {"error": f"Agent B failed: {exc}"})
                return None
            out = str(resp.get("output", ""))
            if resp.get("llm_prompt"):
                run.llm_requests.append({
                    "source": "agent_b", "label": f"turn_{turn}", "prompt": resp["llm_prompt"],
                    "response": resp.get("llm_response"),
                    "endpoint": resp.get("llm_endpoint") or client.llm_url(), "turn": turn,
                    "llm_meta": resp.get("llm_meta") or {}})
            outputs.append(out)
            run.b_outputs.append(out)
            run.ev("agent_b_response", f"Received Agent B response (turn {turn})",
                   tool_call_id=tcid, extra={"turn": turn, "output_preview": out[:200]})
            progress = ("You are Agent A. Provide a short progress check after this turn. "
                        "Summarize what's done, what's unclear, and one next step.\n\n"
                        f"{run.role_block}\nUser task:\n{task}\n\n"
                        f"Agent B notes (turn {turn}):\n{out}\n\n"
                        f"Context so far:\n{context or '(none yet)'}")
            try:
                note = run.llm(f"progress_check_{turn}", progress, "agent_a.progress_check",
                               "sub_call", turn=turn)
                run.notes.append(note)
                run.ev("agent_a_progress_check", f"Progress check completed (turn {turn})",
                       extra={"output_preview": note[:200]})
            except Exception as exc:
                run.ev("agent_a_progress_check_error", f"Progress check failed (turn {turn}): {exc}")
            context = (context + "\n" + out).strip()[-2000:]
        final = ("You are Agent A. The user task is:\n"
                 f"{run.role_block}\n{task}\n\n"
                 "Agent B provided these iterative notes:\n"
                 f"{context}\n\n"
                 "Use the notes to produce the final concise answer. Ignore any progress check "
                 "notes unless useful. Now produce the final concise answer for the user task.")
        return final, "\n---\n".join(outputs)


def run():
    port = env_int("AGENT_A_PORT", 8101)
    serve(AgentAHandler, HOST, port, f"[*] Agent A HTTP server listening on http://{HOST}:{port}/task")


if __name__ == "__main__":
    run()
