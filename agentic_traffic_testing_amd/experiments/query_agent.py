"""Send one request to Agent A (/task) or Agent B (/subtask) and print the JSON reply
(reference scripts/experiment/query_agent.py:1-54)."""
from __future__ import annotations

import argparse
import json
import sys

import httpx

DEFAULT_ENDPOINTS = {"a": "http://localhost:8101/task", "b": "http://localhost:8102/subtask"}


def send(agent: str, text: str, scenario: str | None, url: str, timeout: float = 30.0) -> dict:
    payload = {"task" if agent == "a" else "subtask": text}
    if scenario:
        payload["scenario"] = scenario
    r = httpx.post(url, json=payload, timeout=timeout)
    r.raise_for_status()
    return r.json()


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Send one request to an agent HTTP endpoint")
    ap.add_argument("agent", choices=("a", "b"))
    ap.add_argument("text")
    ap.add_argument("--scenario", default=None)
    ap.add_argument("--url", default=None)
    ap.add_argument("--timeout", type=float, default=30.0)
    a = ap.parse_args(argv)
    print(json.dumps(send(a.agent, a.text, a.scenario, a.url or DEFAULT_ENDPOINTS[a.agent],
                          a.timeout), indent=2))
    return 0


if __name__ == "__main__":
    sys.exit(main())
