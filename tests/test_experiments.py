"""Experiment pipeline (output contract §5.5.7) against a fake
Prometheus and a fake Agent A."""
import csv
import json
import time
import urllib.parse
from datetime import datetime, timedelta, timezone
from pathlib import Path

import numpy as np
import pytest

from agentic_traffic_testing_amd.experiments import (correlate_metrics, iat_stats, plot_results,
                                                     runner, scrape_metrics, supervise)
from agentic_traffic_testing_amd.experiments.prom import PromClient
from agentic_traffic_testing_amd.observability import dashboard

ROOT = Path(__file__).resolve().parents[1]


def fake_prom():
    calls = []

    def fetch(url):
        q = urllib.parse.parse_qs(urllib.parse.urlparse(url).query)
        calls.append(q)
        expr = q["query"][0]
        if "query_range" in url:
            start, end, step = float(q["start"][0]), float(q["end"][0]), float(q["step"][0])
            ts = np.arange(start, end, step)
            if "NOSUCH" in expr:
                return {"status": "error", "error": "bad"}
            vals = [[t, str(1.0 + (i % 3))] for i, t in enumerate(ts)] + [[end, "NaN"]]
            return {"status": "success", "data": {"result": [
                {"metric": {"src_service": "agent_a"}, "values": vals}]}}
        return {"status": "success", "data": {"result": [
            {"metric": {}, "value": [0, "2.5"]}, {"metric": {}, "value": [0, "1.5"]}]}}

    return PromClient("http://prom", fetch=fetch), calls


def test_scrape_metrics_csv(tmp_path):
    client, calls = fake_prom()
    panels = scrape_metrics.dashboard_panels(dashboard.build_dashboard())
    assert panels[0]["row"] == "Overview" and panels[-1]["row"] == "MI355X Engine"
    rows = scrape_metrics.scrape(panels[:3], client, 1_000_000, 1_030_000, 5,
                                 {"task_slug": "t", "task_id": "x", "iteration": 2}, verbose=False)
    n = scrape_metrics.write_csv(rows, tmp_path / "metrics.csv")
    assert n == len(rows) > 0
    with open(tmp_path / "metrics.csv") as f:
        r = list(csv.DictReader(f))
    assert list(r[0].keys()) == scrape_metrics.FIELDNAMES
    assert r[0]["row_section"] == "Overview" and r[0]["task_slug"] == "t"
    assert json.loads(r[0]["labels"]) == {"src_service": "agent_a"}
    assert float(calls[0]["start"][0]) == pytest.approx(1_000_000 / 1000 - 60)
    assert all(row["value"] == row["value"] for row in rows)  # NaN dropped


def _calls_log(path, base):
    recs = []
    for tid, n in (("task-1", 3), ("task-2", 1)):
        for i in range(n):
            t0 = base + timedelta(seconds=5 * i)
            recs.append({"task_id": tid, "agent_id": "AgentA" if i == 0 else "AgentB",
                         "prompt_tokens": 10, "completion_tokens": 5, "total_tokens": 15,
                         "latency_ms": 100, "model_name": "m",
                         "timestamp_start": t0.isoformat(),
                         "timestamp_end": (t0 + timedelta(seconds=2)).isoformat()})
    path.write_text("\n".join(json.dumps(r) for r in recs) + "\nnot json\n")


def test_correlate_metrics(tmp_path, monkeypatch):
    monkeypatch.setenv("COST_PER_INPUT_TOKEN_USD", "0.001")
    monkeypatch.setenv("COST_PER_OUTPUT_TOKEN_USD", "0.002")
    _calls_log(tmp_path / "calls.jsonl", datetime(2026, 1, 1, tzinfo=timezone.utc))
    av = tmp_path / "av"
    av.mkdir()
    (av / "task-1.json").write_text(json.dumps({"task_id": "task-1"}))
    client, calls = fake_prom()
    out = tmp_path / "corr.csv"
    assert correlate_metrics.main(["--call-log", str(tmp_path / "calls.jsonl"),
                                   "--agentverse-dir", str(av), "--output", str(out)],
                                  client=client) == 0
    rows = list(csv.DictReader(open(out)))
    assert [r["task_id"] for r in rows] == ["task-1", "task-2"]
    r1 = rows[0]
    assert list(r1.keys()) == correlate_metrics.FIELDNAMES
    assert r1["total_llm_calls"] == "3" and r1["agent_b_calls"] == "2"
    assert float(r1["window_s"]) == 15.0 and r1["scenario"] == "agentverse"
    assert float(r1["cost_estimate_usd"]) == pytest.approx(30 * 0.001 + 15 * 0.002)
    assert float(r1["tcp_bytes_to_llm"]) == 4.0  # sum over series
    assert float(r1["tcp_rtt_p50_s"]) == 2.5     # first series
    assert any("[15s]" in c["query"][0] for c in calls)


def test_iat_stats():
    rng = np.random.default_rng(0)
    v = rng.exponential(0.5, size=2000)
    d = iat_stats.describe(v)
    assert d["cv"] == pytest.approx(1.0, abs=0.08)
    assert d["lb_p"] > 0.01
    fits = iat_stats.fit(v)
    assert {f["name"] for f in fits} >= {"expon", "gamma", "weibull_min"}
    assert fits[0]["name"] in ("expon", "gamma", "weibull_min")
    # AR(1)-correlated gaps: Ljung-Box must flag dependence
    x = np.empty(500)
    x[0] = 1
    for i in range(1, 500):
        x[i] = 0.8 * x[i - 1] + rng.normal(0, 0.1) + 0.2
    assert iat_stats.ljung_box(np.abs(x), 10)[1] < 1e-6
    assert any("Best-fit by AIC" in ln for ln in iat_stats.report("x", v))


def _fake_agentverse(counter):
    def send(url, task, cfg):
        counter["n"] += 1
        if counter.get("fail_at") == counter["n"]:
            raise RuntimeError("boom")
        now = datetime.now(timezone.utc)
        reqs = [{"source": "agent_a" if i % 2 else "agent-b-1",
                 "start_time_utc": (now + timedelta(milliseconds=137 * i * (1 + i % 3))).isoformat()}
                for i in range(12)]
        return {"task_id": f"tid{counter['n']}", "llm_requests": reqs,
                "iteration_history": [{"evaluation": {"score": 60}}, {"evaluation": {"score": 92}}]}
    return send


def test_experiment_runner_and_resume(tmp_path):
    client, _ = fake_prom()
    out = tmp_path / "exp"
    counter = {"n": 0}
    cfg = runner.Config(out_dir=out, iterations=2, wait_s=0, plots=False)
    ex = runner.Experiment(cfg, send=_fake_agentverse(counter), sleep=lambda s: None, prom=client)
    n_tasks = len(ex.tasks)
    assert [s for s, _ in ex.tasks] == ["mathematical-problem", "research-task",
                                        "software-development", "consulting"]
    assert ex.run() == 0
    runs = runner.read_runs(out / "runs.jsonl")
    assert len(runs) == 2 * n_tasks
    meta = json.loads((Path(runs[0]["run_dir"]) / "meta.json").read_text())
    assert meta["agentverse"]["iteration_scores"] == [60, 92] and meta["iteration"] == 1
    assert (Path(runs[0]["run_dir"]) / "metrics.csv").exists() and (out / "metrics.csv").exists()
    summ = (out / "summary.txt").read_text()
    assert f"--- Run {2 * n_tasks} / {2 * n_tasks}" in summ and "  DONE" in summ

    # crash after 3 runs, then resume with -c -o
    out2 = tmp_path / "exp2"
    c2 = {"n": 0}
    ex2 = runner.Experiment(runner.Config(out_dir=out2, iterations=2, wait_s=0, plots=False),
                            send=_fake_agentverse(c2), sleep=lambda s: None, prom=client)
    orig = ex2.one_run
    state = {"k": 0}

    def crashing(log, st, it, slug, task):
        state["k"] += 1
        if state["k"] > 3:
            raise KeyboardInterrupt
        orig(log, st, it, slug, task)

    ex2.one_run = crashing
    with pytest.raises(KeyboardInterrupt):
        ex2.run()
    assert len(runner.read_runs(out2 / "runs.jsonl")) == 3
    resumed = runner.Experiment(runner.Config(out_dir=out2, resume=True, wait_s=0, plots=False),
                                send=_fake_agentverse(c2), sleep=lambda s: None, prom=client)
    assert resumed.run() == 0
    runs2 = runner.read_runs(out2 / "runs.jsonl")
    assert len(runs2) == 2 * n_tasks
    assert [(r["iteration"], r["task_slug"]) for r in runs2] == [
        (it, s) for it in (1, 2) for s, _ in resumed.tasks]
    assert "RESUMED" in (out2 / "summary.txt").read_text()
    # resuming a finished experiment only finalizes
    again = runner.Experiment(runner.Config(out_dir=out2, resume=True, wait_s=0, plots=False),
                              send=_fake_agentverse(c2), sleep=lambda s: None, prom=client)
    assert again.run() == 0 and len(runner.read_runs(out2 / "runs.jsonl")) == 2 * n_tasks


def test_plot_results_outputs(tmp_path):
    client, _ = fake_prom()
    out = tmp_path / "exp"
    ex = runner.Experiment(runner.Config(out_dir=out, iterations=2, wait_s=0, plots=False),
                           send=_fake_agentverse({"n": 0}), sleep=lambda s: None, prom=client)
    ex.run()
    dash = ROOT / "infra/monitoring/grafana/provisioning/dashboards/agentic-traffic.json"
    files = plot_results.run(out, dash)
    names = {f.name for f in files}
    assert {"01_Overview.png", "08_Traffic_Characterization.png", "interarrival_distribution.png",
            "interarrival_ecdf.png", "per_run_summary.png", "task_comparison_summary.png",
            "interarrival_from_responses.png", "interarrival_fit.png",
            "interarrival_fit_report.txt", "statistics.txt"} <= names
    assert all(f.exists() and f.stat().st_size > 0 for f in files)
    assert "Best-fit by AIC" in (out / "plots" / "interarrival_fit_report.txt").read_text()


def test_supervise_check(tmp_path):
    exp = tmp_path / "exp"
    exp.mkdir()
    (exp / "summary.txt").write_text("...\n  DONE\n")
    state = tmp_path / "state.json"
    state.write_text(json.dumps({"pid": 999999, "experiment_dir": str(exp)}))
    assert supervise.check(state) == 0
    assert not state.exists()
    assert supervise.check(state) == 0  # no state: nothing to do
