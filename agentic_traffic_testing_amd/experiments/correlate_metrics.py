"""Join per-call LLM logs with Prometheus TCP telemetry, one row per task (reference
scripts/experiment/correlate_metrics.py:1-406).

For every ``task_id`` in ``llm_calls.jsonl`` the task window is
[min(timestamp_start), max(timestamp_end)] of its calls (at least ``--min-window-s``);
TCP counters are ``increase()`` instant queries at the window end with the window as the
lookback: bytes / packets agents -> LLM and back, Agent A -> Agent B fan-out, SYN count,
flow-duration and handshake-RTT p50/p95 for agent_a -> llm_backend.  Application fields
are summed from the call records (cost from ``COST_PER_{INPUT,OUTPUT}_TOKEN_USD``);
``scenario`` comes from a persisted AgentVerse record when one exists.

Caveat kept from the reference: Prometheus data is time-windowed, not per task, so
concurrent tasks share TCP attribution - run experiments serially for clean rows.
"""
from __future__ import annotations

import argparse
import csv
import json
import os
import sys
from collections import defaultdict
from datetime import datetime, timezone
from pathlib import Path

from .prom import PromClient

FIELDNAMES = [
    "task_id", "scenario", "task_start", "task_end", "window_s",
    "total_llm_calls", "agent_a_calls", "agent_b_calls",
    "total_prompt_tokens", "total_completion_tokens", "total_tokens",
    "total_llm_latency_ms", "cost_estimate_usd", "model_name",
    "tcp_bytes_to_llm", "tcp_bytes_from_llm", "tcp_packets_to_llm",
    "tcp_bytes_a_to_b", "tcp_packets_a_to_b", "tcp_syn_count",
    "tcp_flow_duration_p50_s", "tcp_flow_duration_p95_s", "tcp_rtt_p50_s", "tcp_rtt_p95_s",
]
TO_LLM = '{src_service=~"agent_a|agent_b.*",dst_service="llm_backend"}'
FROM_LLM = '{src_service="llm_backend",dst_service=~"agent_a|agent_b.*"}'
A_TO_B = '{src_service="agent_a",dst_service=~"agent_b.*"}'
A_LLM = 'src_service="agent_a",dst_service="llm_backend"'


def tcp_queries(window_s: float) -> dict:
    w = f"{max(window_s, 15.0):.0f}s"

    def q(p, metric):
        return (f"histogram_quantile({p}, sum by (le) "
                f"(increase({metric}_bucket{{{A_LLM}}}[{w}])))")

    return {
        "tcp_bytes_to_llm": ("sum", f"sum(increase(tcp_bytes_total{TO_LLM}[{w}]))"),
        "tcp_bytes_from_llm": ("sum", f"sum(increase(tcp_bytes_total{FROM_LLM}[{w}]))"),
        "tcp_packets_to_llm": ("sum", f"sum(increase(tcp_packets_total{TO_LLM}[{w}]))"),
        "tcp_bytes_a_to_b": ("sum", f"sum(increase(tcp_bytes_total{A_TO_B}[{w}]))"),
        "tcp_packets_a_to_b": ("sum", f"sum(increase(tcp_packets_total{A_TO_B}[{w}]))"),
        "tcp_syn_count": ("sum", f"sum(increase(tcp_syn_total[{w}]))"),
        "tcp_flow_duration_p50_s": ("first", q(0.5, "tcp_flow_duration_seconds")),
        "tcp_flow_duration_p95_s": ("first", q(0.95, "tcp_flow_duration_seconds")),
        "tcp_rtt_p50_s": ("first", q(0.5, "tcp_rtt_handshake_seconds")),
        "tcp_rtt_p95_s": ("first", q(0.95, "tcp_rtt_handshake_seconds")),
    }


def query_tcp(client: PromClient, end_s: float, window_s: float) -> dict:
    out = {}
    for k, (kind, expr) in tcp_queries(window_s).items():
        out[k] = client.scalar_sum(expr, end_s) if kind == "sum" else client.first(expr, end_s)
    return out


def load_calls(path: Path) -> dict[str, list[dict]]:
    by_task = defaultdict(list)
    if not path.exists():
        print(f"WARN call log not found: {path}", file=sys.stderr)
        return by_task
    for i, line in enumerate(path.read_text(encoding="utf-8").splitlines(), 1):
        if not line.strip():
            continue
        try:
            rec = json.loads(line)
        except json.JSONDecodeError as e:
            print(f"WARN skipping malformed line {i}: {e}", file=sys.stderr)
            continue
        if rec.get("task_id"):
            by_task[rec["task_id"]].append(rec)
    return by_task


def _ts(v) -> float | None:
    if not v:
        return None
    try:
        return datetime.fromisoformat(str(v).replace("Z", "+00:00")).timestamp()
    except ValueError:
        return None


def task_window(calls: list[dict]) -> tuple[float | None, float | None]:
    starts = [t for t in (_ts(c.get("timestamp_start")) for c in calls) if t is not None]
    ends = [t for t in (_ts(c.get("timestamp_end")) for c in calls) if t is not None]
    return (min(starts), max(ends)) if starts and ends else (None, None)


def load_agentverse(d: Path) -> dict[str, dict]:
    meta = {}
    if d.is_dir():
        for f in d.glob("*.json"):
            try:
                rec = json.loads(f.read_text(encoding="utf-8"))
            except (OSError, json.JSONDecodeError):
                continue
            if isinstance(rec, dict) and rec.get("task_id"):
                meta[rec["task_id"]] = rec
    return meta


def _rate(name: str) -> float:
    try:
        return float(os.environ.get(name, "0") or 0)
    except ValueError:
        return 0.0


def app_row(task_id: str, calls: list[dict], av: dict | None) -> dict:
    pt = sum(c.get("prompt_tokens") or 0 for c in calls)
    ct = sum(c.get("completion_tokens") or 0 for c in calls)
    ri, ro = _rate("COST_PER_INPUT_TOKEN_USD"), _rate("COST_PER_OUTPUT_TOKEN_USD")
    scenario = None
    if av:
        scenario = (av.get("result") or {}).get("scenario") or av.get("scenario") or "agentverse"
    return {"task_id": task_id, "scenario": scenario, "total_llm_calls": len(calls),
            "agent_a_calls": sum(c.get("agent_id") == "AgentA" for c in calls),
            "agent_b_calls": sum(c.get("agent_id") == "AgentB" for c in calls),
            "total_prompt_tokens": pt, "total_completion_tokens": ct,
            "total_tokens": sum(c.get("total_tokens") or 0 for c in calls),
            "total_llm_latency_ms": sum(c.get("latency_ms") or 0 for c in calls),
            "cost_estimate_usd": round(pt * ri + ct * ro, 8) if (ri or ro) else None,
            "model_name": calls[0].get("model_name") if calls else None}


def correlate(calls_by_task: dict, av_meta: dict, client: PromClient,
              min_window_s: float = 15.0) -> list[dict]:
    rows = []
    for tid, calls in sorted(calls_by_task.items()):
        s, e = task_window(calls)
        if s is None:
            print(f"  WARN  skipping {tid[:12]}: no timestamps", file=sys.stderr)
            continue
        w = max(e - s, min_window_s)
        row = app_row(tid, calls, av_meta.get(tid))
        row.update(task_start=datetime.fromtimestamp(s, tz=timezone.utc).isoformat(),
                   task_end=datetime.fromtimestamp(e, tz=timezone.utc).isoformat(),
                   window_s=round(w, 3))
        row.update(query_tcp(client, e, w))
        rows.append(row)
    return rows


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Correlate LLM call logs with TCP telemetry")
    ap.add_argument("--call-log", default="logs/llm_calls.jsonl")
    ap.add_argument("--agentverse-dir", default="logs/agentverse")
    ap.add_argument("--prometheus", default="http://localhost:9090")
    ap.add_argument("--output", default="data/correlated.csv")
    ap.add_argument("--min-window-s", type=float, default=15.0)
    return ap


def main(argv: list[str] | None = None, client: PromClient | None = None) -> int:
    a = build_parser().parse_args(argv)
    calls = load_calls(Path(a.call_log))
    if not calls:
        print("ERROR no task records found in call log.", file=sys.stderr)
        return 1
    rows = correlate(calls, load_agentverse(Path(a.agentverse_dir)),
                     client or PromClient(a.prometheus), a.min_window_s)
    if not rows:
        print("ERROR no rows produced.", file=sys.stderr)
        return 1
    out = Path(a.output)
    out.parent.mkdir(parents=True, exist_ok=True)
    with open(out, "w", newline="", encoding="utf-8") as f:
        w = csv.DictWriter(f, fieldnames=FIELDNAMES, extrasaction="ignore")
        w.writeheader()
        w.writerows(rows)
    print(f"Wrote {len(rows)} rows -> {out}", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
