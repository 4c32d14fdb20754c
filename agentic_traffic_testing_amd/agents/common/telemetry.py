"""JSONL telemetry events (reference agents/common/telemetry.py:1-75).

One JSON object per line in ``logs/<NODE_NAME>_<agent_id>.log`` with the fields
task_id, agent_id, tool_call_id, event_type, message, timestamp_ms, scenario, extra,
node_id (sorted keys) - the format the analysis scripts group by task_id.

Fix vs the reference: the reference shares one logger per handler class and
mutates ``.scenario`` per request, so concurrent requests can log each other's scenario.
Here ``log()`` takes an explicit ``scenario`` override and writes are serialised by a lock,
so the shared logger is safe across request threads.
"""
from __future__ import annotations

import json
import os
import socket
import sys
import threading
import time
import uuid


def now_ms() -> int:
    return int(time.time() * 1000)


def node_id() -> str:
    return os.environ.get("NODE_NAME", socket.gethostname())


class TelemetryLogger:
    _locks: dict[str, threading.Lock] = {}
    _locks_guard = threading.Lock()

    def __init__(self, agent_id: str, log_file: str | None = None, scenario: str | None = None):
        self.agent_id = agent_id
        self.scenario = scenario
        self.node_id = node_id()
        self._fixed_file = log_file

    @property
    def log_file(self) -> str:
        """Resolved per call so TELEMETRY_LOG_DIR changes (tests, stacks) take effect."""
        if self._fixed_file:
            return self._fixed_file
        return os.path.join(os.environ.get("TELEMETRY_LOG_DIR", "logs"),
                            f"{self.node_id}_{self.agent_id}.log")

    @staticmethod
    def _lock_for(path: str) -> threading.Lock:
        with TelemetryLogger._locks_guard:
            lk = TelemetryLogger._locks.get(path)
            if lk is None:
                d = os.path.dirname(path)
                if d:
                    os.makedirs(d, exist_ok=True)
                lk = TelemetryLogger._locks[path] = threading.Lock()
            return lk

    @staticmethod
    def new_task_id() -> str:
        return str(uuid.uuid4())

    @staticmethod
    def new_tool_call_id() -> str:
        return str(uuid.uuid4())

    def log(self, task_id: str, event_type: str, message: str, tool_call_id: str | None = None,
            extra: dict | None = None, scenario: str | None = None) -> dict:
        rec = {
            "task_id": task_id,
            "agent_id": self.agent_id,
            "tool_call_id": tool_call_id,
            "event_type": event_type,
            "message": message,
            "timestamp_ms": now_ms(),
            "scenario": scenario if scenario is not None else self.scenario,
            "extra": extra or {},
            "node_id": self.node_id,
        }
        line = json.dumps(rec, sort_keys=True, default=str)
        path = self.log_file
        try:
            with self._lock_for(os.path.abspath(path)), open(path, "a", encoding="utf-8") as f:
                f.write(line + "\n")
        except OSError as exc:
            print(f"[telemetry-error] {exc}: {line}", file=sys.stderr)
        return rec
