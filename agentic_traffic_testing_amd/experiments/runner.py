"""Repeatable AgentVerse experiment runner with resume (reference
scripts/experiment/run_experiment.sh:1-580, SURVEY §2.2 E1, §3.5, output contract §5.5.7).

For iteration 1..N and every ``example_tasks[]`` entry of
agents/templates/agentverse_workflow.json (slug = lower-cased name with non-alphanumerics
collapsed to ``-``): POST ``/agentverse`` (``stream: false``, 600 s timeout,
``max_iterations`` / ``success_threshold`` from ``AGENTVERSE_*``), save
``<RUN_TS>_<slug>_<task_id>/{response.json, meta.json}``, append to ``runs.jsonl``, wait
``wait_s`` for Prometheus, scrape the run window (step 5).  After the last run the whole
experiment window is scraped (step 15, ``task_slug=all``) and the plots are produced.
Everything printed is tee'd to ``summary.txt``.

Resume (``-c -o DIR``): the position comes from the last record of ``runs.jsonl`` and the
original parameters from ``summary.txt`` ("Iterations :", "--- Run i / n", "Agent A :",
"Prometheus :" - the same lines the reference parses), so a killed run (the supervisor
in ``supervise.py`` restarts it) continues after the last completed task.  A failed
request is reported and skipped, as in the reference.

The HTTP call and the sleeps are injectable so the whole loop is testable in-process.
"""
from __future__ import annotations

import argparse
import json
import re
import sys
import time
from dataclasses import dataclass, field
from datetime import datetime
from pathlib import Path

import httpx

from . import plot_results
from .prom import PromClient
from .scrape_metrics import dashboard_panels, scrape, write_csv

REPO = Path(__file__).resolve().parents[2]
DASHBOARD = REPO / "infra/monitoring/grafana/provisioning/dashboards/agentic-traffic.json"
TEMPLATE = Path(__file__).resolve().parents[1] / "agents/templates/agentverse_workflow.json"


def slugify(name: str) -> str:
    return re.sub(r"[^a-z0-9]+", "-", name.lower()).strip("-")


def load_tasks(template: Path = TEMPLATE) -> list[tuple[str, str]]:
    data = json.loads(Path(template).read_text())
    return [(slugify(t.get("name", "")), t["task"].strip())
            for t in data.get("example_tasks", []) if t.get("task", "").strip()]


def now_ms() -> int:
    return int(time.time() * 1000)


@dataclass
class Config:
    out_dir: Path
    iterations: int = 0
    agent_a_url: str = "http://localhost:8101"
    prometheus_url: str = "http://localhost:9090"
    wait_s: float = 20.0
    max_iterations: int = 3
    success_threshold: int = 90
    dashboard: Path = DASHBOARD
    template: Path = TEMPLATE
    resume: bool = False
    plots: bool = True
    request_timeout_s: float = 600.0


@dataclass
class State:
    start_iter: int = 1
    start_task: int = 0
    run_count: int = 0
    total_runs: int = 0
    experiment_start_ms: int = field(default_factory=now_ms)


class Tee:
    def __init__(self, path: Path):
        self.f = open(path, "a", encoding="utf-8")

    def __call__(self, msg: str = ""):
        print(msg, flush=True)
        self.f.write(msg + "\n")
        self.f.flush()

    def close(self):
        self.f.close()


def parse_summary(path: Path) -> dict:
    out = {"iterations": None, "total_runs": None, "last_run": 0, "agent_a": None,
           "prometheus": None}
    for line in path.read_text(encoding="utf-8").splitlines():
        m = re.match(r"^\s+Iterations\s+:\s+(\d+)", line)
        if m:
            out["iterations"] = int(m.group(1))
        m = re.match(r"^--- Run (\d+) / (\d+)", line)
        if m:
            out["last_run"], out["total_runs"] = int(m.group(1)), int(m.group(2))
        m = re.match(r"^\s+Agent A\s+:\s+(\S+)", line)
        if m and out["agent_a"] is None:
            out["agent_a"] = m.group(1)
        m = re.match(r"^\s+Prometheus\s+:\s+(\S+)", line)
        if m and out["prometheus"] is None:
            out["prometheus"] = m.group(1)
    return out


def read_runs(path: Path) -> list[dict]:
    if not path.exists():
        return []
    return [json.loads(x) for x in path.read_text().splitlines() if x.strip()]


def post_agentverse(url: str, task: str, cfg: Config) -> dict:
    r = httpx.post(url.rstrip("/") + "/agentverse",
                   json={"task": task, "stream": False, "max_iterations": cfg.max_iterations,
                         "success_threshold": cfg.success_threshold},
                   timeout=cfg.request_timeout_s)
    r.raise_for_status()
    return r.json()


class Experiment:
    def __init__(self, cfg: Config, send=post_agentverse, sleep=time.sleep, prom=None):
        self.cfg = cfg
        self.send = send
        self.sleep = sleep
        self.prom = prom or PromClient(cfg.prometheus_url)
        self.tasks = load_tasks(cfg.template)
        self.panels = dashboard_panels(cfg.dashboard) if Path(cfg.dashboard).exists() else []
        self.out = Path(cfg.out_dir)
        self.runs_log = self.out / "runs.jsonl"
        self.summary = self.out / "summary.txt"
        self.failed = 0

    # -------------------------------------------------------------------------------
    def prepare(self, log) -> State | None:
        cfg, n_tasks = self.cfg, len(self.tasks)
        if not cfg.resume:
            st = State(total_runs=cfg.iterations * n_tasks)
            log("=" * 64)
            log("  Agentic Traffic Experiment")
            log(f"  Timestamp  : {datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}")
            log(f"  Iterations : {cfg.iterations} per task ({n_tasks} tasks total)")
            log(f"  Agent A    : {cfg.agent_a_url}")
            log(f"  Prometheus : {cfg.prometheus_url}")
            log(f"  Output     : {self.out}")
            log("=" * 64)
            return st
        info = parse_summary(self.summary)
        runs = read_runs(self.runs_log)
        cfg.iterations = info["iterations"] or cfg.iterations
        if cfg.agent_a_url == Config.agent_a_url and info["agent_a"]:
            cfg.agent_a_url = info["agent_a"]
        if cfg.prometheus_url == Config.prometheus_url and info["prometheus"]:
            cfg.prometheus_url = info["prometheus"]
            self.prom = PromClient(cfg.prometheus_url)
        st = State(total_runs=info["total_runs"] or cfg.iterations * n_tasks,
                   run_count=info["last_run"])
        slugs = [s for s, _ in self.tasks]
        if runs:
            last = runs[-1]
            if last["task_slug"] not in slugs:
                raise SystemExit(f"ERROR: last task '{last['task_slug']}' not in template")
            st.start_iter = int(last["iteration"])
            st.start_task = slugs.index(last["task_slug"]) + 1
            if st.start_task >= n_tasks:
                st.start_iter, st.start_task = st.start_iter + 1, 0
            st.experiment_start_ms = int(runs[0]["run_start_ms"])
            st.run_count = max(st.run_count, len(runs))
        log("")
        log("=" * 64)
        log(f"  RESUMED at {datetime.now().strftime('%Y-%m-%d_%H-%M-%S')}")
        log(f"  Experiment  : {self.out}")
        log(f"  Iterations  : {cfg.iterations} per task ({n_tasks} tasks)")
        log(f"  Total Runs  : {st.total_runs}")
        log(f"  Resuming at : iter={st.start_iter}, task="
            f"{slugs[st.start_task] if st.start_iter <= cfg.iterations else 'none'}")
        log(f"  Agent A     : {cfg.agent_a_url}")
        log(f"  Prometheus  : {cfg.prometheus_url}")
        log("=" * 64)
        return st

    def one_run(self, log, st: State, it: int, slug: str, task: str):
        st.run_count += 1
        run_ts = datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
        t0, start_ms = time.time(), now_ms()
        log("")
        log(f"--- Run {st.run_count} / {st.total_runs}  |  iter={it}  task={slug} ---")
        log(f"  Time  : {run_ts}")
        log(f"  Task  : {task[:80]}...")
        try:
            resp = self.send(self.cfg.agent_a_url, task, self.cfg)
        except Exception as e:  # noqa: BLE001 - a failed run is logged and skipped
            log(f"  ERROR: Request failed: {e}")
            self.failed += 1
            return
        end_ms = now_ms()
        dur = int(time.time() - t0)
        task_id = resp.get("task_id") or resp.get("taskId") or "unknown"
        run_dir = self.out / f"{run_ts}_{slug}_{task_id}"
        run_dir.mkdir(parents=True, exist_ok=True)
        (run_dir / "response.json").write_text(json.dumps(resp, indent=2))
        scores = []
        for h in resp.get("iteration_history") or []:
            try:
                scores.append(int((h.get("evaluation") or {}).get("score")))
            except (TypeError, ValueError):
                scores.append(None)
        meta = {"task": task, "task_slug": slug, "iteration": it, "task_id": task_id,
                "run_ts": run_ts, "run_start_ms": start_ms, "run_end_ms": end_ms,
                "duration_s": dur, "agent_a_url": self.cfg.agent_a_url,
                "prometheus_url": self.cfg.prometheus_url,
                "agentverse": {"max_iterations": self.cfg.max_iterations,
                               "success_threshold": self.cfg.success_threshold,
                               "iteration_scores": scores}}
        (run_dir / "meta.json").write_text(json.dumps(meta, indent=2))
        with open(self.runs_log, "a") as f:
            f.write(json.dumps({"run_dir": str(run_dir), "task_slug": slug, "iteration": it,
                                "task_id": task_id, "run_start_ms": start_ms,
                                "run_end_ms": end_ms, "duration_s": dur}) + "\n")
        log(f"  Task ID  : {task_id}")
        log(f"  Duration : {dur}s")
        log(f"  Saved response -> {run_dir / 'response.json'}")
        log(f"  Waiting {self.cfg.wait_s:g}s for metrics to propagate...")
        self.sleep(self.cfg.wait_s)
        rows = scrape(self.panels, self.prom, start_ms, end_ms, 5,
                      {"task_slug": slug, "task_id": task_id, "iteration": it}, verbose=False)
        write_csv(rows, run_dir / "metrics.csv")
        log(f"  Metrics saved -> {run_dir / 'metrics.csv'} ({len(rows)} rows)")

    def finalize(self, log):
        if self.cfg.plots:
            log("")
            log("Generating plots...")
            try:
                plot_results.run(self.out, Path(self.cfg.dashboard))
                log(f"  Plots saved -> {self.out / 'plots'}/")
            except Exception as e:  # noqa: BLE001
                log(f"  WARNING: Plotting failed: {e}")
        log("")
        log("=" * 64)
        log("  DONE")
        log(f"  Results: {self.out}")
        log("=" * 64)

    def run(self) -> int:
        self.out.mkdir(parents=True, exist_ok=True)
        log = Tee(self.summary)
        try:
            st = self.prepare(log)
            t_start = time.time()
            if st.start_iter > self.cfg.iterations:
                log("")
                log(f"Experiment already complete! All {st.total_runs} runs finished.")
                self.finalize(log)
                return 0
            for it in range(st.start_iter, self.cfg.iterations + 1):
                first = st.start_task if it == st.start_iter else 0
                for slug, task in self.tasks[first:]:
                    self.one_run(log, st, it, slug, task)
            end_ms = now_ms()
            log("")
            log("=" * 64)
            log(f"  All runs complete: {st.run_count} total, {self.failed} failed")
            log(f"  Experiment duration: {int(time.time() - t_start)}s")
            log("  Scraping full experiment window...")
            log("=" * 64)
            rows = scrape(self.panels, self.prom, st.experiment_start_ms, end_ms, 15,
                          {"task_slug": "all", "task_id": "aggregate", "iteration": 0},
                          verbose=False)
            write_csv(rows, self.out / "metrics.csv")
            log(f"  Aggregate metrics saved -> {self.out / 'metrics.csv'} ({len(rows)} rows)")
            self.finalize(log)
            return 0
        finally:
            log.close()


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="AgentVerse traffic experiment runner")
    ap.add_argument("-n", type=int, default=None, help="iterations per task (fresh runs)")
    ap.add_argument("-c", action="store_true", help="continue an interrupted experiment (-o)")
    ap.add_argument("-o", default=None, help="output dir (existing dir with -c)")
    ap.add_argument("-a", default="http://localhost:8101", help="Agent A base URL")
    ap.add_argument("-p", default="http://localhost:9090", help="Prometheus URL")
    ap.add_argument("-w", type=float, default=20.0, help="seconds to wait after each run")
    ap.add_argument("--no-plots", action="store_true")
    ap.add_argument("--template", default=str(TEMPLATE))
    ap.add_argument("--dashboard-json", default=str(DASHBOARD))
    return ap


def main(argv: list[str] | None = None) -> int:
    import os

    a = build_parser().parse_args(argv)
    if a.c:
        if not a.o:
            print("ERROR: -c requires -o <existing-experiment-dir>", file=sys.stderr)
            return 1
        out = Path(a.o)
        for f in ("summary.txt", "runs.jsonl"):
            if not (out / f).exists():
                print(f"ERROR: {f} not found in {out}", file=sys.stderr)
                return 1
    else:
        if not a.n or a.n < 1:
            print("ERROR: -n <iterations> (positive integer) is required, or -c to resume",
                  file=sys.stderr)
            return 1
        out = Path(a.o) if a.o else REPO / "data" / "runs" / (
            "experiment_" + datetime.now().strftime("%Y-%m-%d_%H-%M-%S"))
    cfg = Config(out_dir=out, iterations=a.n or 0, agent_a_url=a.a, prometheus_url=a.p,
                 wait_s=a.w, resume=a.c, plots=not a.no_plots, template=Path(a.template),
                 dashboard=Path(a.dashboard_json),
                 max_iterations=int(os.environ.get("AGENTVERSE_MAX_ITERATIONS", "3")),
                 success_threshold=int(float(os.environ.get("AGENTVERSE_SUCCESS_THRESHOLD",
                                                            "90"))))
    return Experiment(cfg).run()


if __name__ == "__main__":
    sys.exit(main())
