"""Agent A client helpers + standalone CLI (reference agents/agent_a/main.py:1-116).

``call_llm`` / ``call_agent_b`` open a NEW TCP connection per call (module-level
``httpx.post``), which is part of the L4 traffic signature of the /task scenarios.
"""
from __future__ import annotations

import argparse
import json
import os

from ..common.http import env_float, llm_output, post_json_new_conn
from ..common.telemetry import TelemetryLogger


def llm_url() -> str:
    return os.environ.get("LLM_SERVER_URL", "http://localhost:8000/chat")


def agent_b_url() -> str:
    return os.environ.get("AGENT_B_URL", "http://agent-b:8102/subtask")


def agent_b_urls() -> list[str]:
    urls = [u.strip() for u in os.environ.get("AGENT_B_URLS", "").split(",") if u.strip()]
    return urls or [agent_b_url()]


def call_llm(prompt: str, headers: dict | None = None, max_tokens: int | None = None):
    payload = {"prompt": prompt}
    if max_tokens is not None:
        payload["max_tokens"] = max_tokens
    data = post_json_new_conn(llm_url(), payload, headers, env_float("LLM_TIMEOUT_SECONDS", 120.0))
    return llm_output(data)


def call_agent_b(subtask: str, scenario: str | None = None, headers: dict | None = None,
                 agent_b_role: str | None = None, agent_b_contract: str | None = None,
                 agent_b_url_override: str | None = None) -> dict:
    payload = {"subtask": subtask}
    if scenario:
        payload["scenario"] = scenario
    if agent_b_role:
        payload["agent_b_role"] = agent_b_role
    if agent_b_contract:
        payload["agent_b_contract"] = agent_b_contract
    d = post_json_new_conn(agent_b_url_override or agent_b_url(), payload, headers,
                           env_float("AGENT_B_TIMEOUT_SECONDS", 120.0))
    return {"output": str(d.get("output", "")), "llm_prompt": d.get("llm_prompt"),
            "llm_response": d.get("llm_response"), "llm_endpoint": d.get("llm_endpoint"),
            "llm_meta": d.get("llm_meta")}


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="Agent A (standalone)")
    ap.add_argument("task")
    ap.add_argument("--scenario", default=None)
    a = ap.parse_args(argv)
    log = TelemetryLogger(agent_id="AgentA", scenario=a.scenario)
    task_id = log.new_task_id()
    log.log(task_id, "task_received", a.task)
    tcid = log.new_tool_call_id()
    log.log(task_id, "llm_request", "Calling LLM server", tool_call_id=tcid,
            extra={"url": llm_url()})
    out, _ = call_llm(a.task)
    log.log(task_id, "llm_response", "Received LLM response", tool_call_id=tcid,
            extra={"output_preview": out[:200]})
    print(json.dumps({"task_id": task_id, "agent_id": "AgentA", "output": out}))


if __name__ == "__main__":
    main()
