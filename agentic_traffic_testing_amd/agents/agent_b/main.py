"""Agent B client helper + standalone CLI (reference agents/agent_b/main.py:1-68)."""
from __future__ import annotations

import argparse
import json
import os

from ..common.http import env_float, llm_output, post_json_new_conn
from ..common.telemetry import TelemetryLogger

LLM_SERVER_URL = os.environ.get("LLM_SERVER_URL", "http://localhost:8000/chat")
LLM_TIMEOUT_SECONDS = env_float("LLM_TIMEOUT_SECONDS", 120.0)


def call_llm(prompt: str, headers: dict | None = None, url: str | None = None) -> tuple[str, dict]:
    """POST {"prompt"} to the LLM backend on a new connection; returns (output, meta)."""
    data = post_json_new_conn(url or os.environ.get("LLM_SERVER_URL", LLM_SERVER_URL),
                              {"prompt": prompt}, headers,
                              env_float("LLM_TIMEOUT_SECONDS", LLM_TIMEOUT_SECONDS))
    return llm_output(data)


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="Agent B (standalone demo)")
    ap.add_argument("subtask")
    ap.add_argument("--scenario", default=None)
    a = ap.parse_args(argv)
    log = TelemetryLogger(agent_id="AgentB", scenario=a.scenario)
    task_id = log.new_task_id()
    log.log(task_id, "subtask_received", a.subtask)
    tcid = log.new_tool_call_id()
    log.log(task_id, "llm_request", "Calling LLM server from AgentB", tool_call_id=tcid,
            extra={"url": LLM_SERVER_URL})
    out, _ = call_llm(a.subtask)
    log.log(task_id, "llm_response", "AgentB received LLM response", tool_call_id=tcid,
            extra={"output_preview": out[:200]})
    print(json.dumps({"task_id": task_id, "agent_id": "AgentB", "output": out}))


if __name__ == "__main__":
    main()
