"""AgentVerse 4-stage multi-agent workflow (reference agents/agent_a/orchestrator.py).

Loop per iteration (AgentVerse, arXiv 2308.10848): (1) expert recruitment - one LLM call;
(2) collaborative decision - horizontal discussion (each expert speaks in turn through its
Agent B replica, up to 3 rounds, early stop when every expert emits ``[CONSENSUS]``, then a
synthesis LLM call with max_tokens 2048) or vertical (solver proposes, reviewers critique
IN PARALLEL, up to 3 rounds, stop when all ``[APPROVED]``); (3) execution - every expert's
subtask in parallel on its Agent B replica; (4) evaluation - one token-budgeted LLM call
whose score is compared with ``success_threshold`` to decide whether to iterate.  Then a
final synthesis call (max_tokens 4096).

Traffic-relevant behaviour kept from the reference: one persistent ``httpx.Client`` for all
orchestrator calls (keep-alive, unlike the per-call connections of the /task scenarios);
expert i -> ``AGENT_B_URLS[i % n]``; ``X-Request-ID`` / ``X-Task-ID`` / ``traceparent``
headers; sequential horizontal rounds vs parallel review/execution fan-out.

Response and SSE contract: ``WorkflowRunner.run`` returns the reference's
``_state_to_response`` shape; progress events are ``iteration_start``, ``stage_start``,
``stage_complete``, ``llm_request``, ``llm_error``, ``discussion_round``,
``vertical_iteration``, ``execution_result``, ``iteration_complete``, ``workflow_error``.

Fixes / additions:
* ``llm_requests[].seq`` is assigned under a lock (the reference computes it from
  ``len(list)+1`` in parallel threads);
* evaluation budgeting counts tokens with the same tokenizer as the backend (the reference
  needs vLLM for that and otherwise falls back to characters);
* ``AGENTVERSE_ORACLE=1``: with random-init weights no response parses,
  which collapses every run to 1 expert / horizontal / score 0.  The oracle substitutes
  well-formed recruitment and evaluation decisions (seeded by task id) *after* the real LLM
  call, so the request stream keeps its full length while the fan-out shape follows a
  realistic distribution.  Entries record ``oracle: true`` when used.
"""
from __future__ import annotations

import hashlib
import json
import os
import random
import re
import threading
import time
import uuid
from concurrent.futures import ThreadPoolExecutor, as_completed
from dataclasses import dataclass, field
from datetime import datetime, timezone
from enum import Enum
from typing import Any, Callable

import httpx

from ..common import tracing
from ..common.http import env_float, env_int
from ..common.telemetry import TelemetryLogger
from . import prompts as P


def _urls_from_env() -> list[str]:
    urls = [u.strip() for u in os.environ.get("AGENT_B_URLS", "").split(",") if u.strip()]
    return urls or [os.environ.get("AGENT_B_URL", "http://agent-b:8102/subtask")]


class Structure(Enum):
    HORIZONTAL = "horizontal"
    VERTICAL = "vertical"


CommunicationStructure = Structure


@dataclass
class Expert:
    role: str
    responsibilities: str
    contract: str
    endpoint: str | None = None
    index: int = 0


@dataclass
class RecruitmentResult:
    experts: list
    communication_structure: Structure
    execution_order: list
    reasoning: str


@dataclass
class DecisionResult:
    final_decision: str
    discussion_rounds: list
    consensus_reached: bool
    structure_used: str
    solver_role: str | None = None
    reviewer_roles: list = field(default_factory=list)


@dataclass
class ExecutionResult:
    outputs: list
    success_count: int
    failure_count: int


@dataclass
class EvaluationResult:
    goal_achieved: bool
    score: int
    criteria: dict | None = None
    rationale: str | None = None
    feedback: str = ""
    missing_aspects: list = field(default_factory=list)
    should_iterate: bool = False


@dataclass
class AgentVerseState:
    task_id: str
    original_task: str
    iteration: int = 0
    max_iterations: int = 3
    success_threshold: int = 70
    recruitment: RecruitmentResult | None = None
    decision: DecisionResult | None = None
    execution: ExecutionResult | None = None
    evaluation: EvaluationResult | None = None
    iteration_history: list = field(default_factory=list)
    llm_requests: list = field(default_factory=list)
    final_output: str | None = None
    completed: bool = False
    lock: threading.Lock = field(default_factory=threading.Lock, repr=False)


# ---- response parsing ------------------------------------------------------------------
def parse_json_response(text: str, default=None):
    """JSON object from an LLM reply: bare JSON, fenced ```json blocks, or the outermost
    {...} span inside prose."""
    t = (text or "").strip()
    fence = re.match(r"^```(?:json)?\s*(.*?)\s*```$", t, flags=re.S)
    if fence:
        t = fence.group(1).strip()
    try:
        return json.loads(t)
    except (json.JSONDecodeError, ValueError):
        pass
    a, b = t.find("{"), t.rfind("}")
    if a != -1 and b > a:
        try:
            return json.loads(t[a:b + 1])
        except (json.JSONDecodeError, ValueError):
            pass
    return default


def parse_markdown_fields(text: str) -> dict | None:
    """Recover score / goal / iterate / rationale / feedback / missing aspects from a
    Markdown-formatted evaluation reply."""
    t = (text or "").strip()
    if t.startswith("```"):
        t = t.split("\n", 1)[1] if "\n" in t else ""
        t = t.rsplit("```", 1)[0]

    def grab(pat):
        m = re.search(pat, t, flags=re.I | re.M)
        return m.group(1).strip() if m else None

    def as_bool(v):
        if v is None:
            return None
        return {"yes": True, "true": True, "no": False, "false": False}.get(v.lower())

    out: dict = {}
    s = grab(r"score\s*[:\-]\s*([0-9]{1,3})")
    if s is not None:
        out["score"] = max(0, min(100, int(s)))
    g = as_bool(grab(r"goal(?:\s+achieved)?\s*[:\-]\s*(yes|no|true|false)"))
    if g is not None:
        out["goal_achieved"] = g
    it = as_bool(grab(r"should\s*iterate\s*[:\-]\s*(yes|no|true|false)"))
    if it is not None:
        out["should_iterate"] = it
    for key in ("rationale", "feedback"):
        v = grab(rf"{key}\s*[:\-]\s*(.+)")
        if v:
            out[key] = v
    m = re.search(r"(?:missing\s+aspects?|gaps?|areas\s+for\s+improvement)\s*[:\-]?\s*\n"
                  r"((?:\s*[-*]\s+.+\n?)+)", t, flags=re.I)
    if m:
        items = [ln.strip().lstrip("-*").strip() for ln in m.group(1).splitlines()]
        items = [i for i in items if i]
        if items:
            out["missing_aspects"] = items
    return out or None


# ---- oracle (random-weights mode) --------------------------------------------------------
ORACLE_ROLES = [
    ("planner", "Break the task into an ordered plan"),
    ("researcher", "Collect the facts and background the task needs"),
    ("executor", "Carry out the concrete steps and computations"),
    ("critic", "Find errors, gaps and risks in the work"),
    ("summarizer", "Condense the results into a clear answer"),
]
assert tuple(r for r, _ in ORACLE_ROLES) == P.ROLES  # the recruitment prompt's vocabulary


def oracle_recruitment(task_id: str, iteration: int, max_experts: int) -> dict:
    rng = random.Random(hashlib.sha256(f"{task_id}:{iteration}:r".encode()).hexdigest())
    n = rng.randint(min(3, max_experts), max(min(3, max_experts), max_experts))
    roles = ORACLE_ROLES[:]
    rng.shuffle(roles)
    picked = sorted(roles[:n], key=lambda r: [x[0] for x in ORACLE_ROLES].index(r[0]))
    structure = "vertical" if rng.random() < 0.5 else "horizontal"
    return {
        "experts": [{"role": r, "responsibilities": d,
                     "contract": f"You are the {r}. {d}. Stay within your role."}
                    for r, d in picked],
        "communication_structure": structure,
        "execution_order": [r for r, _ in picked],
        "reasoning": f"oracle: {n} experts, {structure} structure",
    }


def oracle_evaluation(task_id: str, iteration: int, threshold: int = 80) -> dict:
    """Seeded evaluator reply in the EVALUATION_PROMPT schema: criteria 0-100, overall score
    = their weighted average with the prompt's weights (30/30/15/15/10)."""
    rng = random.Random(hashlib.sha256(f"{task_id}:{iteration}:e".encode()).hexdigest())
    crit = {k: rng.randint(50, 100) for k in P.CRITERIA_WEIGHTS}
    score = int(round(sum(P.CRITERIA_WEIGHTS[k] * v for k, v in crit.items())))
    ok = score >= threshold
    return {"goal_achieved": ok, "score": score, "criteria": crit,
            "rationale": "oracle: weighted average of seeded criterion scores "
                         "(completeness 30%, correctness 30%, clarity 15%, relevance 15%, "
                         "actionability 10%)",
            "feedback": "" if ok else "Tighten correctness and cover missing steps.",
            "missing_aspects": [] if ok else ["verification of results"],
            "should_iterate": not ok}


class AgentVerseOrchestrator:
    def __init__(self, logger: TelemetryLogger, tracer=None,
                 progress_callback: Callable[[dict], None] | None = None,
                 http_client: httpx.Client | None = None):
        self.logger = logger
        self.tracer = tracer or tracing.get_tracer("agent-a-orchestrator")
        self.progress_callback = progress_callback
        self.llm_url = os.environ.get("LLM_SERVER_URL", "http://localhost:8000/chat")
        self.llm_timeout = env_float("LLM_TIMEOUT_SECONDS", 120.0)
        self.b_timeout = env_float("AGENT_B_TIMEOUT_SECONDS", 120.0)
        self.max_workers = env_int("MAX_PARALLEL_WORKERS", 5)
        self.agent_b_urls = _urls_from_env()
        self.max_model_len = env_int("LLM_MAX_MODEL_LEN", 4096)
        self.max_tokens = env_int("LLM_MAX_TOKENS", 512)
        self.eval_max_tokens = env_int("LLM_EVAL_MAX_TOKENS", self.max_tokens)
        self.margin = env_int("LLM_PROMPT_SAFETY_MARGIN_TOKENS", 128)
        self.eval_max_chars = env_int("EVAL_MAX_PROMPT_CHARS", 20000)
        self.oracle = os.environ.get("AGENTVERSE_ORACLE", "0").lower() in ("1", "true", "yes")
        self.http = http_client or httpx.Client(timeout=self.llm_timeout)
        self._tok = None

    # ---- transport -------------------------------------------------------------------------
    def _progress(self, event: str, data: dict):
        if self.progress_callback:
            self.progress_callback({"event": event, "data": data})

    def _call_llm(self, prompt: str, headers: dict | None = None, max_tokens: int | None = None):
        payload: dict[str, Any] = {"prompt": prompt}
        if max_tokens is not None:
            payload["max_tokens"] = max_tokens
        with self.tracer.start_as_current_span("agent_a.call_llm",
                                               kind=tracing.SpanKind.CLIENT) as sp:
            sp.set_attribute("app.request_start_time_utc", _utc())
            sp.set_attribute("app.llm.url", self.llm_url)
            if max_tokens is not None:
                sp.set_attribute("llm.max_tokens", int(max_tokens))
            hdr = tracing.inject(dict(headers or {}))
            r = self.http.post(self.llm_url, json=payload, headers=hdr, timeout=self.llm_timeout)
            r.raise_for_status()
            data = r.json()
            meta = data.get("meta") if isinstance(data.get("meta"), dict) else {}
            return str(data.get("output", "")), {
                "llm_backend": meta,
                "otel": {"agent_a": tracing.span_to_metadata(sp),
                         "llm_backend": meta.get("otel", {})}}

    def _call_agent_b(self, subtask: str, expert: Expert, headers: dict, task_id: str) -> dict:
        url = expert.endpoint or self.agent_b_urls[0]
        if not isinstance(url, str) or not url.strip():
            raise ValueError(f"Invalid Agent B URL: {url!r}")
        self.logger.log(task_id, "agent_b_call_attempt", f"Calling Agent B at {url}",
                        extra={"url": url, "role": expert.role, "scenario": "agentic_verse"},
                        scenario="agentic_verse")
        payload = {"subtask": subtask, "scenario": "agentic_verse",
                   "agent_b_role": expert.role}
        if expert.contract:
            payload["agent_b_contract"] = expert.contract
        try:
            r = self.http.post(url, json=payload, headers=headers, timeout=self.b_timeout)
            r.raise_for_status()
            d = r.json()
        except httpx.ConnectError as e:
            msg = (f"Failed to connect to Agent B at {url}. Error: {e}. Available URLs: "
                   f"{self.agent_b_urls}")
            self.logger.log(task_id, "agent_b_connection_error", msg,
                            extra={"url": url, "role": expert.role}, scenario="agentic_verse")
            raise ConnectionError(msg) from e
        except httpx.TimeoutException as e:
            msg = f"Timeout connecting to Agent B at {url} (timeout: {self.b_timeout}s)"
            self.logger.log(task_id, "agent_b_timeout_error", msg,
                            extra={"url": url, "role": expert.role}, scenario="agentic_verse")
            raise TimeoutError(msg) from e
        except httpx.HTTPStatusError as e:
            msg = (f"Agent B returned error status {e.response.status_code} for URL {url}: "
                   f"{e.response.text[:200]}")
            self.logger.log(task_id, "agent_b_http_error", msg,
                            extra={"url": url, "status_code": e.response.status_code},
                            scenario="agentic_verse")
            raise
        return {"output": str(d.get("output", "")), "llm_prompt": d.get("llm_prompt"),
                "llm_response": d.get("llm_response"), "llm_endpoint": d.get("llm_endpoint"),
                "llm_meta": d.get("llm_meta") if isinstance(d.get("llm_meta"), dict) else None,
                "otel": d.get("otel") if isinstance(d.get("otel"), dict) else None}

    # ---- request log -----------------------------------------------------------------------
    def _record(self, st: AgentVerseState, *, stage: str, label: str, prompt: str,
                response: str, source: str = "Agent A", agent_role: str | None = None,
                endpoint: str | None = None, round_num: int | None = None,
                duration_seconds: float | None = None, request_id: str | None = None,
                otel: dict | None = None, llm_meta: dict | None = None,
                start_time_utc: str | None = None, error: bool = False, oracle: bool = False):
        role = agent_role if agent_role is not None else (
            "orchestrator" if source == "Agent A" else None)
        with st.lock:
            entry: dict[str, Any] = {
                "seq": len(st.llm_requests) + 1, "iteration": st.iteration, "stage": stage,
                "label": label, "source": source, "prompt": prompt, "response": response,
                "endpoint": endpoint or self.llm_url, "error": error}
            for k, v in (("start_time_utc", start_time_utc), ("request_id", request_id),
                         ("otel", otel), ("llm_meta", llm_meta), ("agent_role", role),
                         ("round", round_num)):
                if v is not None:
                    entry[k] = v
            if duration_seconds is not None:
                entry["duration_seconds"] = round(duration_seconds, 2)
            if oracle:
                entry["oracle"] = True
            st.llm_requests.append(entry)
        self._progress("llm_error" if error else "llm_request", entry)

    def _llm_tracked(self, st: AgentVerseState, prompt: str, stage: str, label: str,
                     max_tokens: int | None = None) -> str:
        rid = str(uuid.uuid4())[:8]
        headers = {"X-Request-ID": rid, "X-Task-ID": st.task_id}
        t0 = time.time()
        start = _utc(t0)
        try:
            out, meta = self._call_llm(prompt, headers=headers, max_tokens=max_tokens)
        except Exception as exc:
            detail = str(exc)
            resp = getattr(exc, "response", None)
            if resp is not None:
                try:
                    detail = resp.json().get("error", detail)
                except Exception:
                    pass
            self._record(st, stage=stage, label=label, prompt=prompt,
                         response=f"[LLM ERROR: {detail}]", duration_seconds=time.time() - t0,
                         request_id=rid, llm_meta={"error": detail}, start_time_utc=start,
                         error=True)
            raise
        self._record(st, stage=stage, label=label, prompt=prompt, response=out,
                     duration_seconds=time.time() - t0, request_id=rid, otel=meta.get("otel"),
                     llm_meta=meta.get("llm_backend"), start_time_utc=start)
        return out

    def _agent_b_tracked(self, st: AgentVerseState, expert: Expert, prompt: str, stage: str,
                         label: str, round_num: int | None = None) -> tuple[str, bool]:
        rid = str(uuid.uuid4())[:8]
        headers = tracing.inject({"X-Request-ID": rid, "X-Task-ID": st.task_id})
        t0 = time.time()
        start = _utc(t0)
        src = f"agent-b-{expert.index + 1}"
        try:
            r = self._call_agent_b(prompt, expert, headers, st.task_id)
        except Exception as exc:
            out = f"[Agent error: {exc}]"
            self._record(st, stage=stage, label=label, prompt=prompt, response=out, source=src,
                         agent_role=expert.role, round_num=round_num,
                         duration_seconds=time.time() - t0, request_id=rid,
                         start_time_utc=start, error=True)
            return out, False
        out = r.get("output", "")
        self._record(st, stage=stage, label=label, prompt=r.get("llm_prompt") or prompt,
                     response=r.get("llm_response") or out, source=src, agent_role=expert.role,
                     endpoint=r.get("llm_endpoint"), round_num=round_num,
                     duration_seconds=time.time() - t0, request_id=rid, otel=r.get("otel"),
                     llm_meta=r.get("llm_meta"), start_time_utc=start)
        return out, True

    # ---- stage 1 -----------------------------------------------------------------------------
    def recruit_experts(self, st: AgentVerseState, feedback: str | None = None) -> RecruitmentResult:
        with self.tracer.start_as_current_span("orchestrator.recruit_experts") as span:
            span.set_attribute("app.task_id", st.task_id)
            span.set_attribute("app.iteration", st.iteration)
            self._progress("stage_start", {"stage": "recruitment", "stage_number": 1,
                                           "iteration": st.iteration,
                                           "message": "Analyzing task and recruiting expert agents..."})
            fb = f"\nFeedback from previous iteration:\n{feedback}\n" if feedback else ""
            self.logger.log(st.task_id, "agentverse_recruitment_start", "Starting expert recruitment",
                            extra={"iteration": st.iteration}, scenario="agentic_verse")
            resp = self._llm_tracked(st, P.RECRUITMENT.format(task=st.original_task,
                                                               feedback_context=fb),
                                     "recruitment", "expert_recruitment")
            parsed = parse_json_response(resp, {})
            if not isinstance(parsed, dict) or not parsed.get("experts"):
                parsed = (parse_markdown_fields(resp) or {}) if not isinstance(parsed, dict) or not parsed else parsed
            used_oracle = False
            if self.oracle and not parsed.get("experts"):
                parsed = oracle_recruitment(st.task_id, st.iteration, self.max_workers)
                used_oracle = True
                st.llm_requests[-1]["oracle"] = True
            experts = []
            for i, e in enumerate((parsed.get("experts") or [])[:self.max_workers]):
                if not isinstance(e, dict):
                    continue
                ep = self.agent_b_urls[i % len(self.agent_b_urls)]
                experts.append(Expert(role=str(e.get("role", "executor")),
                                      responsibilities=str(e.get("responsibilities", "")),
                                      contract=str(e.get("contract", "")), endpoint=ep,
                                      index=len(experts)))
            if not experts:
                experts = [Expert("executor", "Execute the given task",
                                  "You are an executor agent. Complete the assigned task thoroughly.",
                                  self.agent_b_urls[0], 0)]
            try:
                structure = Structure(str(parsed.get("communication_structure",
                                                     "horizontal")).lower())
            except ValueError:
                structure = Structure.HORIZONTAL
            reasoning = str(parsed.get("reasoning", "") or "").strip() or (
                f"Selected {structure.value} communication structure with {len(experts)} "
                f"expert(s): {', '.join(e.role for e in experts)}.")
            order = parsed.get("execution_order")
            res = RecruitmentResult(experts, structure,
                                    order if isinstance(order, list) else [e.role for e in experts],
                                    reasoning)
            self.logger.log(st.task_id, "agentverse_recruitment_complete",
                            f"Recruited {len(experts)} experts",
                            extra={"experts": [e.role for e in experts],
                                   "expert_endpoints": {e.role: e.endpoint for e in experts},
                                   "structure": structure.value, "reasoning": reasoning,
                                   "oracle": used_oracle},
                            scenario="agentic_verse")
            span.set_attribute("app.expert_count", len(experts))
            span.set_attribute("app.communication_structure", structure.value)
            self._progress("stage_complete", {
                "stage": "recruitment", "stage_number": 1, "iteration": st.iteration,
                "experts": [{"role": e.role, "responsibilities": e.responsibilities} for e in experts],
                "communication_structure": structure.value, "reasoning": reasoning})
            return res

    # ---- stage 2 -----------------------------------------------------------------------------
    def collaborative_decision(self, st: AgentVerseState, rec: RecruitmentResult) -> DecisionResult:
        with self.tracer.start_as_current_span("orchestrator.collaborative_decision") as span:
            span.set_attribute("app.task_id", st.task_id)
            span.set_attribute("app.structure", rec.communication_structure.value)
            self._progress("stage_start", {
                "stage": "decision", "stage_number": 2, "iteration": st.iteration,
                "message": f"Starting {rec.communication_structure.value} decision-making...",
                "structure": rec.communication_structure.value})
            self.logger.log(st.task_id, "agentverse_decision_start",
                            f"Starting {rec.communication_structure.value} decision-making",
                            scenario="agentic_verse")
            res = (self._horizontal(st, rec) if rec.communication_structure == Structure.HORIZONTAL
                   else self._vertical(st, rec))
            self._progress("stage_complete", {
                "stage": "decision", "stage_number": 2, "iteration": st.iteration,
                "consensus_reached": res.consensus_reached, "structure": res.structure_used,
                "rounds": len(res.discussion_rounds)})
            return res

    def _horizontal(self, st: AgentVerseState, rec: RecruitmentResult, max_rounds: int = 3):
        rounds, history, consensus = [], "", False
        for rn in range(1, max_rounds + 1):
            responses, all_ok = [], True
            for ex in rec.experts:  # sequential: each expert sees the transcript so far
                prompt = P.HORIZONTAL_DISCUSSION.format(
                    role=ex.role, contract=ex.contract, task=st.original_task,
                    discussion_history=history or "(No discussion yet)", round_num=rn)
                out, _ = self._agent_b_tracked(st, ex, prompt, "decision",
                                               f"horizontal_discussion_round{rn}", rn)
                ok = "[CONSENSUS]" in out
                all_ok &= ok
                responses.append({"expert": ex.role, "index": ex.index, "response": out,
                                  "consensus": ok})
            history += f"\n--- Round {rn} ---\n" + "".join(
                f"{r['expert'].upper()}: {r['response']}\n" for r in responses)
            rounds.append({"round": rn, "responses": responses})
            self.logger.log(st.task_id, "agentverse_discussion_round",
                            f"Completed discussion round {rn}",
                            extra={"round": rn, "all_consensus": all_ok}, scenario="agentic_verse")
            self._progress("discussion_round", {"stage": "decision", "round": rn,
                                                "iteration": st.iteration,
                                                "responses": responses, "consensus": all_ok})
            if all_ok:
                consensus = True
                break
        decision = self._llm_tracked(st, P.SYNTHESIZE_DISCUSSION.format(
            task=st.original_task, discussion_history=history), "decision",
            "synthesize_discussion", max_tokens=2048)
        return DecisionResult(decision, rounds, consensus, "horizontal", None,
                              [e.role for e in rec.experts])

    def _vertical(self, st: AgentVerseState, rec: RecruitmentResult, max_rounds: int = 3):
        exs = rec.experts
        solver = next((e for e in exs if e.role == "planner"), exs[0] if exs else None)
        if solver is None:
            return DecisionResult("No solver agent available", [], False, "vertical", None, [])
        reviewers = [e for e in exs if e is not solver]
        rounds, proposal, critiques, approved = [], "", "", True
        ctx = tracing.get_current()
        for it in range(1, max_rounds + 1):
            sp = P.VERTICAL_SOLVER.format(
                contract=solver.contract, task=st.original_task,
                previous_proposal=f"\nYour previous proposal:\n{proposal}\n" if proposal else "",
                critiques=f"\nReviewer critiques:\n{critiques}\n" if critiques else "")
            proposal, ok = self._agent_b_tracked(st, solver, sp, "decision",
                                                 f"vertical_solver_iter{it}", it)
            if not ok:
                proposal = proposal.replace("[Agent error:", "[Solver error:", 1)
            reviews = []
            if reviewers:
                def review(rv: Expert, prop=proposal, rnd=it):
                    tok = tracing.attach(ctx)
                    try:
                        rp = P.VERTICAL_REVIEWER.format(role=rv.role, contract=rv.contract,
                                                        task=st.original_task, proposal=prop)
                        crit, ok2 = self._agent_b_tracked(st, rv, rp, "decision",
                                                          f"vertical_reviewer_{rv.role}_iter{rnd}", rnd)
                        if not ok2:
                            crit = crit.replace("[Agent error:", "[Reviewer error:", 1)
                    finally:
                        tracing.detach(tok)
                    return {"reviewer": rv.role, "critique": crit, "approved": "[APPROVED]" in crit}

                with ThreadPoolExecutor(max_workers=len(reviewers)) as pool:
                    reviews = list(pool.map(review, reviewers))  # keep reviewer order
                approved = all(r["approved"] for r in reviews)
            critiques = "\n".join(f"{r['reviewer']}: {r['critique']}" for r in reviews)
            rounds.append({"iteration": it, "proposal": proposal, "reviewer_responses": reviews,
                           "all_approved": approved})
            self.logger.log(st.task_id, "agentverse_vertical_iteration",
                            f"Completed vertical iteration {it}",
                            extra={"iteration": it, "all_approved": approved},
                            scenario="agentic_verse")
            self._progress("vertical_iteration", {
                "stage": "decision", "iteration": st.iteration, "solver_iteration": it,
                "proposal": proposal[:200] + "..." if len(proposal) > 200 else proposal,
                "reviewer_responses": reviews, "all_approved": approved})
            if approved:
                break
        return DecisionResult(proposal, rounds, approved if reviewers else True, "vertical",
                              solver.role, [r.role for r in reviewers])

    # ---- stage 3 -----------------------------------------------------------------------------
    def execute_actions(self, st: AgentVerseState, rec: RecruitmentResult,
                        dec: DecisionResult) -> ExecutionResult:
        with self.tracer.start_as_current_span("orchestrator.execute_actions") as span:
            span.set_attribute("app.task_id", st.task_id)
            self._progress("stage_start", {
                "stage": "execution", "stage_number": 3, "iteration": st.iteration,
                "message": f"Executing tasks with {len(rec.experts)} agents...",
                "expert_count": len(rec.experts)})
            self.logger.log(st.task_id, "agentverse_execution_start", "Starting action execution",
                            scenario="agentic_verse")
            ctx = tracing.get_current()

            def run(ex: Expert):
                tok = tracing.attach(ctx)
                subtask = (f"Based on your role as {ex.role}:\nResponsibilities: "
                           f"{ex.responsibilities}\n\nExecute your part of the plan:\n"
                           f"{dec.final_decision}\n\nFocus on what is relevant to your expertise.\n")
                try:
                    with self.tracer.start_as_current_span(
                            f"orchestrator.execute_subtask.{ex.role}", kind=tracing.SpanKind.CLIENT):
                        if not ex.endpoint:
                            self.logger.log(st.task_id, "agentverse_execution_error",
                                            f"Expert {ex.role} has no endpoint",
                                            scenario="agentic_verse")
                            raise ValueError(f"Expert {ex.role} has invalid endpoint")
                        prompt = P.EXECUTION.format(role=ex.role, contract=ex.contract,
                                                    task=st.original_task, subtask=subtask,
                                                    decision_context=dec.final_decision[:500])
                        out, ok = self._agent_b_tracked(st, ex, prompt, "execution",
                                                        f"execute_{ex.role}")
                        if not ok:
                            out = out.replace("[Agent error:", "Execution failed:", 1).rstrip("]")
                        return {"expert": ex.role, "index": ex.index, "subtask": subtask,
                                "output": out, "success": ok}
                except Exception as exc:
                    return {"expert": ex.role, "index": ex.index, "subtask": subtask,
                            "output": f"Execution failed: {exc}", "success": False}
                finally:
                    tracing.detach(tok)

            outputs, ok_n, bad_n = [], 0, 0
            with ThreadPoolExecutor(max_workers=max(1, len(rec.experts))) as pool:
                futs = [pool.submit(run, ex) for ex in rec.experts]
                for f in as_completed(futs):
                    r = f.result()
                    outputs.append(r)
                    ok_n += int(r["success"])
                    bad_n += int(not r["success"])
                    self._progress("execution_result", {
                        "stage": "execution", "iteration": st.iteration, "expert": r["expert"],
                        "success": r["success"], "output_preview": r["output"][:200],
                        "completed": len(outputs), "total": len(rec.experts)})
            self.logger.log(st.task_id, "agentverse_execution_complete",
                            f"Execution complete: {ok_n} success, {bad_n} failures",
                            extra={"success": ok_n, "failures": bad_n}, scenario="agentic_verse")
            self._progress("stage_complete", {"stage": "execution", "stage_number": 3,
                                              "iteration": st.iteration, "success_count": ok_n,
                                              "failure_count": bad_n, "total": len(outputs)})
            return ExecutionResult(outputs, ok_n, bad_n)

    # ---- stage 4 -----------------------------------------------------------------------------
    def _count_tokens(self, text: str) -> int:
        if self._tok is None:
            from ...engine.tokenizer import get_tokenizer

            self._tok = get_tokenizer(os.environ.get("LLM_MODEL"))
        return len(self._tok.encode(text))

    def build_evaluation_prompt(self, st: AgentVerseState, results: str, span=None):
        """Token-budgeted evaluation prompt: keep the newest results so the prompt fits
        max_model_len - eval_max_tokens - margin; falls back to a character budget."""
        def render(res):
            return P.EVALUATION.format(task=st.original_task, iteration=st.iteration + 1,
                                       max_iterations=st.max_iterations, results=res,
                                       success_threshold=st.success_threshold)
        budget = self.max_model_len - self.eval_max_tokens - self.margin
        prompt = render(results)
        truncated, trimmed, final_tokens = False, None, None
        try:
            n = self._count_tokens(prompt)
            if budget > 0 and n > budget:
                overhead = self._count_tokens(render(""))
                keep = max(0, budget - overhead)
                ids = self._tok.encode(results)
                trimmed = max(0, len(ids) - keep)
                results = self._tok.decode(ids[trimmed:])
                prompt = render(results)
                truncated = True
            final_tokens = self._count_tokens(prompt)
        except Exception:
            if len(prompt) > self.eval_max_chars:
                over = len(prompt) - self.eval_max_chars
                prompt = render(results[over:])
                truncated = True
        if span is not None:
            span.set_attribute("app.evaluation_prompt_truncated", truncated)
            if trimmed is not None:
                span.set_attribute("app.evaluation_trimmed_tokens", trimmed)
            if final_tokens is not None:
                span.set_attribute("app.evaluation_prompt_tokens", final_tokens)
            span.set_attribute("app.evaluation_token_budget", budget)
        return prompt, truncated, trimmed, final_tokens

    def evaluate_results(self, st: AgentVerseState, ex: ExecutionResult) -> EvaluationResult:
        with self.tracer.start_as_current_span("orchestrator.evaluate_results") as span:
            span.set_attribute("app.task_id", st.task_id)
            span.set_attribute("app.iteration", st.iteration)
            self._progress("stage_start", {
                "stage": "evaluation", "stage_number": 4, "iteration": st.iteration,
                "message": "Evaluating results and determining if iteration is needed..."})
            self.logger.log(st.task_id, "agentverse_evaluation_start", "Starting evaluation",
                            scenario="agentic_verse")
            results = "\n\n".join(f"[{o['expert']}]:\n{o['output']}" for o in ex.outputs)
            prompt, truncated, trimmed, ntok = self.build_evaluation_prompt(st, results, span)
            resp = self._llm_tracked(st, prompt, "evaluation", "evaluate_results",
                                     max_tokens=self.eval_max_tokens)
            parsed = parse_json_response(resp, None)
            if not isinstance(parsed, dict):
                parsed = parse_markdown_fields(resp) or {}
            if self.oracle and "score" not in parsed:
                parsed = oracle_evaluation(st.task_id, st.iteration, st.success_threshold or 80)
                st.llm_requests[-1]["oracle"] = True
            try:
                score = max(0, min(100, int(parsed.get("score"))))
            except (TypeError, ValueError):
                score = 0
            goal = bool(parsed.get("goal_achieved", False))
            iterate = bool(parsed.get("should_iterate", False))
            if st.success_threshold > 0:  # threshold overrides the evaluator's own flags
                goal = score >= st.success_threshold
                iterate = not goal
            if st.iteration + 1 >= st.max_iterations or goal:
                iterate = False
            feedback = str(parsed.get("feedback", "") or "")
            missing = parsed.get("missing_aspects") or []
            rationale = parsed.get("rationale")
            if not feedback.strip() and (iterate or not goal):
                parts = []
                if rationale:
                    parts.append(f"Previous rationale: {rationale}")
                if missing:
                    parts.append(f"Missing or weak aspects: {', '.join(map(str, missing))}.")
                if not parts:
                    parts.append(f"Score {score}/100 is below the acceptance threshold of "
                                 f"{st.success_threshold}. Refine the team composition and "
                                 "instructions so the next iteration closes the gaps.")
                feedback = " ".join(parts)
            if truncated:
                note = ("[System] Evaluation input was truncated to respect the model's "
                        "context window." + (f" Approximately {trimmed} earlier result tokens "
                                             f"were dropped; final prompt is ~{ntok} tokens."
                                             if trimmed is not None else ""))
                feedback = f"{feedback}\n{note}".strip()
            res = EvaluationResult(goal, score, parsed.get("criteria"), rationale, feedback,
                                   missing, iterate)
            self.logger.log(st.task_id, "agentverse_evaluation_complete",
                            f"Evaluation complete: score={score}",
                            extra={"score": score, "goal_achieved": goal,
                                   "should_iterate": iterate}, scenario="agentic_verse")
            self._progress("stage_complete", {
                "stage": "evaluation", "stage_number": 4, "iteration": st.iteration,
                "goal_achieved": goal, "score": score, "criteria": res.criteria,
                "rationale": rationale, "feedback": feedback, "should_iterate": iterate})
            return res

    # ---- workflow ----------------------------------------------------------------------------
    def run_workflow(self, task: str, task_id: str, max_iterations: int = 3,
                     success_threshold: int = 70) -> dict:
        with self.tracer.start_as_current_span("orchestrator.run_workflow") as span:
            span.set_attribute("app.task_id", task_id)
            span.set_attribute("app.success_threshold", success_threshold)
            st = AgentVerseState(task_id, task, max_iterations=max_iterations,
                                 success_threshold=min(100, max(0, success_threshold)))
            self.logger.log(task_id, "agentverse_workflow_start", "Starting AgentVerse workflow",
                            extra={"max_iterations": max_iterations}, scenario="agentic_verse")
            feedback, error = None, None
            try:
                while st.iteration < st.max_iterations:
                    t0 = time.time()
                    self._progress("iteration_start", {
                        "iteration": st.iteration, "max_iterations": st.max_iterations,
                        "message": f"Starting iteration {st.iteration + 1} of {st.max_iterations}..."})
                    st.recruitment = self.recruit_experts(st, feedback)
                    st.decision = self.collaborative_decision(st, st.recruitment)
                    st.execution = self.execute_actions(st, st.recruitment, st.decision)
                    st.evaluation = self.evaluate_results(st, st.execution)
                    ev = st.evaluation
                    st.iteration_history.append({
                        "iteration": st.iteration, "duration_seconds": round(time.time() - t0, 2),
                        "recruitment": {"experts": [e.role for e in st.recruitment.experts],
                                        "structure": st.recruitment.communication_structure.value},
                        "decision": {"consensus": st.decision.consensus_reached,
                                     "rounds": len(st.decision.discussion_rounds)},
                        "execution": {"success": st.execution.success_count,
                                      "failures": st.execution.failure_count},
                        "evaluation": {"goal_achieved": ev.goal_achieved, "score": ev.score,
                                       "criteria": ev.criteria, "rationale": ev.rationale,
                                       "feedback": ev.feedback or ""}})
                    self._progress("iteration_complete", {"iteration_history": st.iteration_history})
                    if not ev.should_iterate:
                        break
                    feedback = ev.feedback
                    st.iteration += 1
                self._progress("stage_start", {"stage": "synthesis", "stage_number": 5,
                                               "iteration": st.iteration,
                                               "message": "Generating final synthesized output..."})
                st.final_output = self._final_output(st)
                st.completed = True
                self._progress("stage_complete", {"stage": "synthesis", "stage_number": 5,
                                                  "iteration": st.iteration,
                                                  "final_output": st.final_output})
                self.logger.log(task_id, "agentverse_workflow_complete",
                                "AgentVerse workflow complete",
                                extra={"iterations": st.iteration + 1,
                                       "final_score": st.evaluation.score if st.evaluation else 0},
                                scenario="agentic_verse")
            except Exception as exc:
                error = str(exc)
                span.set_attribute("app.workflow_error", error)
                self.logger.log(task_id, "agentverse_workflow_error", f"Workflow aborted: {error}",
                                scenario="agentic_verse")
                self._progress("workflow_error", {
                    "error": error, "completed_llm_calls": len(st.llm_requests),
                    "failed_calls": sum(1 for r in st.llm_requests if r.get("error"))})
            out = self.state_to_response(st)
            if error is not None:
                out["workflow_error"] = error
                out["partial"] = True
            return out

    def _final_output(self, st: AgentVerseState) -> str:
        if not st.execution:
            return "No execution results available."
        results = "\n\n".join(f"[{o['expert']}]:\n{o['output']}" for o in st.execution.outputs)
        its = "\n".join(f"Iteration {h['iteration'] + 1}: score={h['evaluation']['score']}, "
                        f"experts={h['recruitment']['experts']}" for h in st.iteration_history)
        ev = st.evaluation
        evaluation = (f"\nScore: {ev.score}/100\nGoal Achieved: {ev.goal_achieved}\n"
                      f"Feedback: {ev.feedback}\n") if ev else ""
        return self._llm_tracked(st, P.FINAL_SYNTHESIS.format(
            task=st.original_task, iteration_summary=its or "(Single iteration)",
            results=results, evaluation=evaluation), "synthesis", "final_output", max_tokens=4096)

    @staticmethod
    def state_to_response(st: AgentVerseState) -> dict:
        rec, dec, ex, ev = st.recruitment, st.decision, st.execution, st.evaluation
        return {
            "task_id": st.task_id,
            "original_task": st.original_task,
            "completed": st.completed,
            "iterations": st.iteration + 1,
            "duration_seconds": sum(h.get("duration_seconds", 0) for h in st.iteration_history),
            "final_output": st.final_output,
            "stages": {
                "recruitment": {
                    "experts": [{"role": e.role, "responsibilities": e.responsibilities,
                                 "endpoint": e.endpoint} for e in (rec.experts if rec else [])],
                    "communication_structure": rec.communication_structure.value if rec else None,
                    "reasoning": rec.reasoning if rec else ""},
                "decision": {
                    "final_decision": dec.final_decision if dec else "",
                    "consensus_reached": dec.consensus_reached if dec else False,
                    "structure_used": dec.structure_used if dec else "",
                    "discussion_rounds": dec.discussion_rounds if dec else [],
                    "solver_role": dec.solver_role if dec else None,
                    "reviewer_roles": dec.reviewer_roles if dec else []},
                "execution": {
                    "outputs": ex.outputs if ex else [],
                    "success_count": ex.success_count if ex else 0,
                    "failure_count": ex.failure_count if ex else 0},
                "evaluation": {
                    "goal_achieved": ev.goal_achieved if ev else False,
                    "score": ev.score if ev else 0,
                    "criteria": ev.criteria if ev else None,
                    "rationale": ev.rationale if ev else None,
                    "feedback": ev.feedback if ev else "",
                    "missing_aspects": ev.missing_aspects if ev else []},
            },
            "iteration_history": st.iteration_history,
            "llm_requests": st.llm_requests,
        }


def _utc(t: float | None = None) -> str:
    return datetime.fromtimestamp(t if t is not None else time.time(), tz=timezone.utc).isoformat()
