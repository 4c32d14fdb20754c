"""Dashboard-driven Prometheus scraper (reference scripts/experiment/scrape_metrics.py:1-281,
SURVEY §2.2 E2, output contract §5.5.7).

The PromQL list is read from the Grafana dashboard JSON, so editing the dashboard changes
what the next experiment records.  Panels are walked in grid order (y, x); a row panel
sets the ``row_section`` of the panels after it.  Every target is range-queried over the
run window widened by 60 s on both sides; rows go to ``metrics.csv`` with the fixed
column order ``FIELDNAMES``.  Queries run on a small thread pool (the reference issues
them one by one); row order stays panel order.
"""
from __future__ import annotations

import argparse
import csv
import json
import sys
from concurrent.futures import ThreadPoolExecutor
from datetime import datetime, timezone
from pathlib import Path

from .prom import PromClient

FIELDNAMES = ["panel_id", "panel_title", "panel_type", "row_section", "unit", "ref_id",
              "legend_format", "expr", "labels", "timestamp", "datetime", "value",
              "task_slug", "task_id", "iteration"]
WINDOW_PAD_MS = 60_000


def dashboard_panels(dashboard: dict | str | Path) -> list[dict]:
    if not isinstance(dashboard, dict):
        dashboard = json.loads(Path(dashboard).read_text())
    raw = sorted(dashboard.get("panels", []),
                 key=lambda p: (p.get("gridPos", {}).get("y", 0), p.get("gridPos", {}).get("x", 0)))
    out, row = [], "General"
    for p in raw:
        if p.get("type") == "row":
            row = p.get("title", "General")
            continue
        targets = [{"refId": t.get("refId", "A"), "expr": t.get("expr", "").strip(),
                    "legendFormat": t.get("legendFormat", "")}
                   for t in p.get("targets", []) if t.get("expr", "").strip()]
        if targets:
            out.append({"id": p.get("id"), "title": p.get("title", f"Panel {p.get('id')}"),
                        "type": p.get("type", ""), "row": row, "gridPos": p.get("gridPos", {}),
                        "unit": p.get("fieldConfig", {}).get("defaults", {}).get("unit", "short"),
                        "targets": targets})
    return out


def scrape(panels: list[dict], client: PromClient, start_ms: int, end_ms: int, step_s: int,
           meta: dict, workers: int = 8, verbose: bool = True) -> list[dict]:
    start_s = (start_ms - WINDOW_PAD_MS) / 1000.0
    end_s = (end_ms + WINDOW_PAD_MS) / 1000.0
    jobs = [(p, t) for p in panels for t in p["targets"]]
    with ThreadPoolExecutor(max(1, workers)) as ex:
        results = list(ex.map(lambda pt: client.range(pt[1]["expr"], start_s, end_s, step_s),
                              jobs))
    rows = []
    for (p, t), series_list in zip(jobs, results):
        if verbose:
            print(f"  scraping  [{p['row']}] {p['title']} {t['refId']}", file=sys.stderr)
        for s in series_list:
            labels = json.dumps(s["labels"], sort_keys=True)
            for ts, v in s["values"]:
                rows.append({
                    "panel_id": p["id"], "panel_title": p["title"], "panel_type": p["type"],
                    "row_section": p["row"], "unit": p["unit"], "ref_id": t["refId"],
                    "legend_format": t["legendFormat"], "expr": t["expr"], "labels": labels,
                    "timestamp": ts,
                    "datetime": datetime.fromtimestamp(ts, tz=timezone.utc).strftime(
                        "%Y-%m-%dT%H:%M:%S.%fZ"),
                    "value": v, **meta})
    return rows


def write_csv(rows: list[dict], path: Path) -> int:
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", newline="", encoding="utf-8") as f:
        w = csv.DictWriter(f, fieldnames=FIELDNAMES, extrasaction="ignore")
        w.writeheader()
        w.writerows(rows)
    return len(rows)


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Scrape Prometheus using a Grafana dashboard's queries")
    ap.add_argument("--dashboard-json", required=True)
    ap.add_argument("--output-dir", required=True)
    ap.add_argument("--prometheus-url", default="http://localhost:9090")
    ap.add_argument("--start-ms", required=True, type=int)
    ap.add_argument("--end-ms", required=True, type=int)
    ap.add_argument("--step", default=5, type=int)
    ap.add_argument("--task-slug", default="unknown")
    ap.add_argument("--task-id", default="unknown")
    ap.add_argument("--iteration", default=0, type=int)
    ap.add_argument("--workers", default=8, type=int)
    return ap


def main(argv: list[str] | None = None, client: PromClient | None = None) -> int:
    a = build_parser().parse_args(argv)
    panels = dashboard_panels(a.dashboard_json)
    print(f"  loaded    {len(panels)} panels from {a.dashboard_json}", file=sys.stderr)
    rows = scrape(panels, client or PromClient(a.prometheus_url), a.start_ms, a.end_ms, a.step,
                  {"task_slug": a.task_slug, "task_id": a.task_id, "iteration": a.iteration},
                  a.workers)
    out = Path(a.output_dir) / "metrics.csv"
    n = write_csv(rows, out)
    print(f"  written   {n} rows -> {out}", file=sys.stderr)
    if n == 0:
        print("  WARN  no data rows scraped - is Prometheus reachable?", file=sys.stderr)
    return 0  # non-fatal either way: the run's response JSON is still saved


if __name__ == "__main__":
    sys.exit(main())
