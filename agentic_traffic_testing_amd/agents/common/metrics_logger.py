"""Per-LLM-call JSONL records in ``logs/llm_calls.jsonl`` (reference
agents/common/metrics_logger.py:1-72; consumed by experiments/correlate_metrics.py).

Record: call_id, task_id, agent_id, parent_call_id, call_type (root | sub_call |
tool_call | verification), prompt_tokens, completion_tokens, total_tokens, latency_ms,
model_name, timestamp_start, timestamp_end, http_status, error.  Token/latency fields come
from the LLM backend's ``meta`` object.
"""
from __future__ import annotations

import json
import os
import sys
import threading
import uuid

CALL_TYPES = ("root", "sub_call", "tool_call", "verification")


class MetricsLogger:
    _lock = threading.Lock()

    def __init__(self, log_dir: str | None = None):
        self._fixed_dir = log_dir

    @property
    def log_file(self) -> str:
        d = self._fixed_dir or os.environ.get("METRICS_LOG_DIR", "logs")
        return os.path.join(d, "llm_calls.jsonl")

    @property
    def model_name(self) -> str:
        return os.environ.get("MODEL_NAME", "unknown")

    def log_call(self, *, task_id: str, agent_id: str, call_type: str, timestamp_start: str,
                 timestamp_end: str, http_status: int, llm_meta: dict | None = None,
                 error: str | None = None, parent_call_id: str | None = None,
                 call_id: str | None = None) -> str:
        meta = llm_meta if isinstance(llm_meta, dict) else {}
        cid = call_id or meta.get("request_id") or str(uuid.uuid4())
        rec = {
            "call_id": cid,
            "task_id": task_id,
            "agent_id": agent_id,
            "parent_call_id": parent_call_id,
            "call_type": call_type,
            "prompt_tokens": meta.get("prompt_tokens"),
            "completion_tokens": meta.get("completion_tokens"),
            "total_tokens": meta.get("total_tokens"),
            "latency_ms": meta.get("latency_ms"),
            "model_name": self.model_name,
            "timestamp_start": timestamp_start,
            "timestamp_end": timestamp_end,
            "http_status": http_status,
            "error": error,
        }
        line = json.dumps(rec, sort_keys=True, default=str)
        path = self.log_file
        try:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            with self._lock, open(path, "a", encoding="utf-8") as f:
                f.write(line + "\n")
        except OSError as exc:
            print(f"[metrics-logger-error] {exc}: {line}", file=sys.stderr)
        return cid
