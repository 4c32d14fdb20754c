"""Experiment plots + statistics (reference scripts/experiment/plot_results.py:1-1290, SURVEY
§2.2 E3, output contract §5.5.7).

Inputs: ``<exp>/metrics.csv`` (aggregate window) and ``<exp>/<run>/metrics.csv`` (per run,
tagged with task_slug / iteration), ``<exp>/<run>/{meta,response}.json``, and the Grafana
dashboard (panel layout, units, row sections).  Outputs under ``<exp>/plots/``:

* ``NN_<Row_Title>.png`` - one figure per dashboard row, one axis per panel
  (time series per target/label set; stat panels as last-value bars);
* ``interarrival_distribution.png`` / ``interarrival_ecdf.png`` - the
  "LLM Interarrival Time (30s rolling avg)" panel per task (time series, histogram + KDE,
  ECDF with p50/p95 markers);
* ``per_run_summary.png`` - run duration and AgentVerse iteration scores per run;
* ``task_comparison_summary.png`` - per-task duration / latency / TTFT / LLM-call counts;
* ``interarrival_from_responses.png`` - inter-arrival times of the LLM requests recorded in
  every response.json (server perspective, per task and per source), independent of
  Prometheus;
* ``interarrival_fit.png`` + ``interarrival_fit_report.txt`` - distribution fits, KS,
  AIC/BIC, CV, ACF and Ljung-Box (``iat_stats``);
* ``statistics.txt`` - per-task summary of the key panels.

White background as the reference actually renders (its docstring says dark - Appendix B).
"""
from __future__ import annotations

import argparse
import json
import re
import sys
from collections import defaultdict
from datetime import datetime
from pathlib import Path

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
from scipy import stats as st  # noqa: E402

from . import iat_stats  # noqa: E402
from .scrape_metrics import dashboard_panels  # noqa: E402

IAT_TITLE = "LLM Interarrival Time (30s rolling avg)"
KEY_PANELS = [IAT_TITLE, "LLM End-to-end Latency (p50/p95)",
              "LLM Time-to-First-Token (TTFT p50/p95)", "In-flight LLM Requests",
              "LLM Request Rate — success vs error"]
PALETTE = ["#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2",
           "#7f7f7f", "#bcbd22", "#17becf"]
UNIT_LABEL = {"s": "seconds", "Bps": "bytes/s", "pps": "packets/s", "bytes": "bytes",
              "percentunit": "fraction", "short": ""}


def _style():
    plt.rcParams.update({"figure.facecolor": "white", "axes.facecolor": "#f7f7f7",
                         "axes.grid": True, "grid.color": "#cccccc", "font.size": 8})


def load_csv(path: Path) -> pd.DataFrame:
    if not path.exists() or path.stat().st_size == 0:
        return pd.DataFrame()
    df = pd.read_csv(path)
    if not df.empty:
        df["timestamp"] = pd.to_numeric(df["timestamp"], errors="coerce")
        df["value"] = pd.to_numeric(df["value"], errors="coerce")
    return df


def load_runs(exp: Path) -> pd.DataFrame:
    parts = [load_csv(d / "metrics.csv") for d in sorted(exp.iterdir())
             if d.is_dir() and d.name != "plots"]
    parts = [p for p in parts if not p.empty]
    return pd.concat(parts, ignore_index=True) if parts else pd.DataFrame()


def _slug(title: str, idx: int) -> str:
    return f"{idx:02d}_" + re.sub(r"[^A-Za-z0-9]+", "_", title).strip("_")


def _series_label(row) -> str:
    leg = str(row.get("legend_format") or "")
    try:
        labels = json.loads(row.get("labels") or "{}")
    except (TypeError, json.JSONDecodeError):
        labels = {}
    if leg and leg != "nan":
        return re.sub(r"\{\{\s*(\w+)\s*\}\}", lambda m: str(labels.get(m.group(1), "")), leg)
    return ",".join(f"{k}={v}" for k, v in sorted(labels.items()) if k != "__name__") or \
        str(row.get("ref_id", ""))


def plot_section(title: str, panels: list[dict], df: pd.DataFrame, out: Path, idx: int) -> Path:
    n = len(panels)
    cols = 2 if n > 1 else 1
    rows = (n + cols - 1) // cols
    fig, axes = plt.subplots(rows, cols, figsize=(7 * cols, 3.2 * rows), squeeze=False)
    fig.suptitle(title, fontsize=12, fontweight="bold")
    for ax, p in zip(axes.flat, panels):
        ax.set_title(p["title"], loc="left", fontsize=9)
        ax.set_ylabel(UNIT_LABEL.get(p["unit"], p["unit"]))
        sub = df[df["panel_title"] == p["title"]] if not df.empty else df
        if sub.empty:
            ax.text(0.5, 0.5, "no data", ha="center", va="center", transform=ax.transAxes,
                    color="#888888")
            continue
        if p["type"] == "stat":
            last = sub.sort_values("timestamp").groupby(["ref_id", "labels"]).tail(1)
            names = [_series_label(r) for _, r in last.iterrows()]
            ax.bar(range(len(last)), last["value"].values,
                   color=PALETTE[:len(last)] if len(last) <= len(PALETTE) else None)
            ax.set_xticks(range(len(last)), names, rotation=20, ha="right", fontsize=7)
            continue
        for i, ((_, _), g) in enumerate(sub.groupby(["ref_id", "labels"], sort=True)):
            g = g.sort_values("timestamp")
            t0 = sub["timestamp"].min()
            ax.plot(g["timestamp"] - t0, g["value"], color=PALETTE[i % len(PALETTE)],
                    linewidth=1.1, label=_series_label(g.iloc[0]))
        ax.set_xlabel("seconds since window start")
        if ax.get_legend_handles_labels()[0]:
            ax.legend(fontsize=6, loc="upper right")
    for ax in list(axes.flat)[n:]:
        ax.axis("off")
    fig.tight_layout()
    path = out / f"{_slug(title, idx)}.png"
    fig.savefig(path, bbox_inches="tight")
    plt.close(fig)
    return path


def plot_interarrival(df: pd.DataFrame, out: Path) -> list[Path]:
    sub = df[df["panel_title"] == IAT_TITLE].dropna(subset=["value"]) if not df.empty else df
    if sub.empty:
        print("  WARN  no interarrival panel data - skipping distribution plots")
        return []
    sub = sub[np.isfinite(sub["value"])]
    tasks = sorted(sub["task_slug"].dropna().astype(str).unique()) or ["all"]
    get = (lambda t: sub[sub["task_slug"].astype(str) == t]) if "task_slug" in sub else (lambda t: sub)
    fig, (a, b) = plt.subplots(1, 2, figsize=(14, 5))
    fig.suptitle("LLM Interarrival Time Distribution", fontsize=12, fontweight="bold")
    a.set_title("Interarrival Time over Experiment", loc="left")
    b.set_title("Distribution (histogram + KDE)", loc="left")
    for i, t in enumerate(tasks):
        g = get(t).sort_values("timestamp")
        c = PALETTE[i % len(PALETTE)]
        a.plot(g["timestamp"] - sub["timestamp"].min(), g["value"], color=c, label=t)
        v = g["value"].values
        if len(v) >= 2:
            b.hist(v, bins=30, density=True, alpha=0.45, color=c, label=f"{t} (n={len(v)})")
            if len(v) > 10 and np.std(v) > 0:
                xs = np.linspace(v.min(), v.max(), 300)
                b.plot(xs, st.gaussian_kde(v)(xs), color=c, linewidth=2)
    a.set_ylabel("seconds")
    b.set_xlabel("interarrival time (s)")
    a.legend(fontsize=7)
    b.legend(fontsize=7)
    fig.tight_layout()
    p1 = out / "interarrival_distribution.png"
    fig.savefig(p1, bbox_inches="tight")
    plt.close(fig)

    fig, ax = plt.subplots(figsize=(8, 5))
    ax.set_title("Interarrival Time - Empirical CDF", loc="left", fontweight="bold")
    ax.set_xlabel("interarrival time (s)")
    ax.set_ylabel("P(X <= x)")
    ax.set_ylim(0, 1.05)
    for i, t in enumerate(tasks):
        v = np.sort(get(t)["value"].values)
        if len(v) < 2:
            continue
        c = PALETTE[i % len(PALETTE)]
        ax.plot(v, np.arange(1, len(v) + 1) / len(v), color=c, linewidth=2,
                label=f"{t} (n={len(v)})")
        for pct, ls in ((50, "--"), (95, ":")):
            pv = np.percentile(v, pct)
            ax.axvline(pv, color=c, linestyle=ls, alpha=0.6)
            ax.text(pv, 0.02 + 0.06 * i, f"p{pct}={pv:.2f}s", color=c, fontsize=6)
    ax.legend(fontsize=8)
    fig.tight_layout()
    p2 = out / "interarrival_ecdf.png"
    fig.savefig(p2, bbox_inches="tight")
    plt.close(fig)
    return [p1, p2]


def run_metas(exp: Path) -> list[dict]:
    metas = []
    for d in sorted(exp.iterdir()):
        m = d / "meta.json"
        if d.is_dir() and m.exists():
            try:
                rec = json.loads(m.read_text())
                rec["_dir"] = d.name
                metas.append(rec)
            except json.JSONDecodeError:
                continue
    return metas


def plot_per_run(exp: Path, out: Path) -> Path | None:
    metas = run_metas(exp)
    if not metas:
        print("  WARN  no run meta.json files - skipping per-run summary")
        return None
    fig, (a, b) = plt.subplots(1, 2, figsize=(14, 4.5))
    fig.suptitle("Per-run summary", fontsize=12, fontweight="bold")
    labels = [f"{m.get('task_slug', '?')}#{m.get('iteration', '?')}" for m in metas]
    dur = [float(m.get("duration_s") or 0) for m in metas]
    colors = {s: PALETTE[i % len(PALETTE)]
              for i, s in enumerate(sorted({m.get("task_slug", "?") for m in metas}))}
    a.bar(range(len(metas)), dur, color=[colors[m.get("task_slug", "?")] for m in metas])
    a.set_xticks(range(len(metas)), labels, rotation=45, ha="right", fontsize=6)
    a.set_ylabel("run duration (s)")
    a.set_title("Run duration", loc="left")
    for i, m in enumerate(metas):
        scores = (m.get("agentverse") or {}).get("iteration_scores") or []
        if scores:
            b.plot(range(1, len(scores) + 1), scores, marker="o", color=colors[m.get("task_slug", "?")],
                   alpha=0.7, label=labels[i])
    b.set_title("AgentVerse evaluation score per iteration", loc="left")
    b.set_xlabel("workflow iteration")
    b.set_ylabel("score")
    if b.get_legend_handles_labels()[0]:
        b.legend(fontsize=6, ncol=2)
    fig.tight_layout()
    p = out / "per_run_summary.png"
    fig.savefig(p, bbox_inches="tight")
    plt.close(fig)
    return p


def plot_task_comparison(exp: Path, df: pd.DataFrame, out: Path) -> Path | None:
    metas = run_metas(exp)
    if not metas:
        return None
    by = defaultdict(lambda: {"dur": [], "calls": []})
    for m in metas:
        slug = m.get("task_slug", "?")
        by[slug]["dur"].append(float(m.get("duration_s") or 0))
        resp = exp / m["_dir"] / "response.json"
        if resp.exists():
            try:
                by[slug]["calls"].append(len(json.loads(resp.read_text()).get("llm_requests", [])))
            except json.JSONDecodeError:
                pass
    tasks = sorted(by)

    def panel_mean(title, ref="A"):
        if df.empty or "task_slug" not in df:
            return [float("nan")] * len(tasks)
        res = []
        for t in tasks:
            s = df[(df["panel_title"] == title) & (df["task_slug"].astype(str) == t)
                   & (df["ref_id"] == ref)]["value"]
            s = s[np.isfinite(s)]
            res.append(float(s.mean()) if len(s) else float("nan"))
        return res

    fig, axes = plt.subplots(1, 4, figsize=(18, 4.2))
    fig.suptitle("Task comparison", fontsize=12, fontweight="bold")
    series = [("mean run duration (s)", [np.mean(by[t]["dur"]) for t in tasks]),
              ("mean LLM calls / run", [np.mean(by[t]["calls"]) if by[t]["calls"] else 0
                                       for t in tasks]),
              ("E2E latency p50 (s)", panel_mean("LLM End-to-end Latency (p50/p95)")),
              ("TTFT p50 (s)", panel_mean("LLM Time-to-First-Token (TTFT p50/p95)"))]
    for ax, (name, vals) in zip(axes, series):
        ax.bar(range(len(tasks)), vals, color=PALETTE[:len(tasks)])
        ax.set_xticks(range(len(tasks)), tasks, rotation=30, ha="right", fontsize=7)
        ax.set_title(name, loc="left")
    fig.tight_layout()
    p = out / "task_comparison_summary.png"
    fig.savefig(p, bbox_inches="tight")
    plt.close(fig)
    return p


def arrivals_from_responses(exp: Path):
    by_task, by_source, all_ts = defaultdict(list), defaultdict(list), []
    for d in sorted(exp.iterdir()):
        resp = d / "response.json"
        if not (d.is_dir() and resp.exists()):
            continue
        slug = None
        if (d / "meta.json").exists():
            try:
                slug = json.loads((d / "meta.json").read_text()).get("task_slug")
            except json.JSONDecodeError:
                pass
        slug = slug or d.name
        try:
            data = json.loads(resp.read_text())
        except json.JSONDecodeError:
            continue
        for req in data.get("llm_requests", []):
            ts = req.get("start_time_utc")
            if not ts:
                continue
            try:
                t = datetime.fromisoformat(str(ts).replace("Z", "+00:00")).timestamp()
            except ValueError:
                continue
            by_task[slug].append(t)
            by_source[req.get("source", "unknown")].append(t)
            all_ts.append(t)
    for dct in (by_task, by_source):
        for k in dct:
            dct[k].sort()
    all_ts.sort()
    return dict(by_task), dict(by_source), all_ts


def plot_iat_from_responses(exp: Path, out: Path) -> Path | None:
    by_task, by_source, all_ts = arrivals_from_responses(exp)
    if len(all_ts) < 2:
        print("  WARN  no response.json llm_requests - skipping response-based IAT plot")
        return None
    fig, axes = plt.subplots(1, 3, figsize=(18, 4.5))
    fig.suptitle("LLM request inter-arrival times (from response.json)", fontsize=12,
                 fontweight="bold")
    iat_all = np.diff(all_ts)
    axes[0].hist(iat_all, bins=40, color=PALETTE[0], alpha=0.7)
    axes[0].set_title(f"All requests, server view (n={len(iat_all)})", loc="left")
    axes[0].set_xlabel("seconds")
    for i, (k, ts) in enumerate(sorted(by_task.items())):
        if len(ts) >= 2:
            v = np.sort(np.diff(ts))
            axes[1].plot(v, np.arange(1, len(v) + 1) / len(v), color=PALETTE[i % len(PALETTE)],
                         label=f"{k} (n={len(v)})")
    axes[1].set_title("ECDF per task", loc="left")
    axes[1].legend(fontsize=6)
    for i, (k, ts) in enumerate(sorted(by_source.items())):
        if len(ts) >= 2:
            v = np.sort(np.diff(ts))
            axes[2].plot(v, np.arange(1, len(v) + 1) / len(v), color=PALETTE[i % len(PALETTE)],
                         label=f"{k} (n={len(v)})")
    axes[2].set_title("ECDF per source", loc="left")
    axes[2].legend(fontsize=6)
    fig.tight_layout()
    p = out / "interarrival_from_responses.png"
    fig.savefig(p, bbox_inches="tight")
    plt.close(fig)
    return p


def analyse_iat(exp: Path, out: Path) -> list[Path]:
    by_task, _, all_ts = arrivals_from_responses(exp)
    if len(all_ts) < 5:
        print("  WARN  too few arrivals for distribution fitting")
        return []
    groups = {"all (server view)": np.diff(all_ts)}
    groups.update({f"task {k}": np.diff(v) for k, v in sorted(by_task.items()) if len(v) >= 5})
    lines = ["Inter-arrival time distribution analysis", "=" * 72]
    for name, vals in groups.items():
        vals = vals[vals > 0]
        if len(vals) >= 3:
            lines += iat_stats.report(name, vals) + [""]
    rep = out / "interarrival_fit_report.txt"
    rep.write_text("\n".join(lines) + "\n")
    v = groups["all (server view)"]
    v = v[v > 0]
    fits = iat_stats.fit(v)
    fig, (a, b) = plt.subplots(1, 2, figsize=(14, 5))
    fig.suptitle("Inter-arrival fit (all requests)", fontsize=12, fontweight="bold")
    a.hist(v, bins=40, density=True, alpha=0.4, color="#888888", label=f"data (n={len(v)})")
    xs = np.linspace(max(v.min(), 1e-6), v.max(), 400) if len(v) else np.array([])
    for i, f in enumerate(fits):
        a.plot(xs, getattr(st, f["name"]).pdf(xs, *f["params"]), color=PALETTE[i],
               label=f"{f['label']} AIC={f['aic']:.0f}")
    a.legend(fontsize=7)
    a.set_xlabel("seconds")
    if fits:
        best = fits[0]
        (osm, osr), _ = st.probplot(v, dist=getattr(st, best["name"]), sparams=best["params"])
        b.plot(osm, osr, "o", ms=3, color=PALETTE[0])
        lim = [min(osm.min(), osr.min()), max(osm.max(), osr.max())]
        b.plot(lim, lim, "--", color="#444444")
        b.set_title(f"Q-Q vs best fit: {best['label']}", loc="left")
    fig.tight_layout()
    p = out / "interarrival_fit.png"
    fig.savefig(p, bbox_inches="tight")
    plt.close(fig)
    return [rep, p]


def statistics_table(df: pd.DataFrame, out: Path) -> Path:
    lines = ["=" * 72, "  Experiment Statistics", "=" * 72]
    for title in KEY_PANELS:
        sub = df[df["panel_title"] == title] if not df.empty else df
        if sub.empty:
            continue
        lines.append(f"\n  {title}")
        tasks = sorted(sub["task_slug"].dropna().astype(str).unique()) if "task_slug" in sub else []
        for t in tasks:
            v = sub[sub["task_slug"].astype(str) == t]["value"].dropna()
            v = v[np.isfinite(v)]
            if len(v):
                lines.append(f"    {t:20s}  n={len(v):4d}  mean={v.mean():8.3f}  "
                             f"p50={v.quantile(0.5):8.3f}  p95={v.quantile(0.95):8.3f}  "
                             f"max={v.max():8.3f}")
    lines.append("\n" + "=" * 72)
    text = "\n".join(lines)
    print(text)
    p = out / "statistics.txt"
    p.write_text(text + "\n")
    return p


def run(exp: Path, dashboard_json: Path) -> list[Path]:
    _style()
    plots = exp / "plots"
    plots.mkdir(exist_ok=True)
    panels = dashboard_panels(dashboard_json)
    df_agg = load_csv(exp / "metrics.csv")
    df_runs = load_runs(exp)
    df = pd.concat([d for d in (df_agg, df_runs) if not d.empty], ignore_index=True) \
        if not (df_agg.empty and df_runs.empty) else pd.DataFrame()
    written = []
    sections = defaultdict(list)
    for p in panels:
        sections[p["row"]].append(p)
    for i, (title, ps) in enumerate(sections.items(), 1):
        written.append(plot_section(title, ps, df, plots, i))
    written += plot_interarrival(df, plots)
    for p in (plot_per_run(exp, plots), plot_task_comparison(exp, df, plots),
              plot_iat_from_responses(exp, plots)):
        if p:
            written.append(p)
    written += analyse_iat(exp, plots)
    written.append(statistics_table(df, plots))
    return written


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Plot experiment metrics like the Grafana dashboard")
    ap.add_argument("--experiment-dir", required=True)
    ap.add_argument("--dashboard-json",
                    default="infra/monitoring/grafana/provisioning/dashboards/agentic-traffic.json")
    a = ap.parse_args(argv)
    exp = Path(a.experiment_dir)
    if not exp.exists():
        print(f"ERROR: experiment-dir does not exist: {exp}", file=sys.stderr)
        return 1
    if not Path(a.dashboard_json).exists():
        print(f"ERROR: dashboard JSON not found: {a.dashboard_json}", file=sys.stderr)
        return 1
    files = run(exp, Path(a.dashboard_json))
    print(f"\n  {len(files)} outputs in {exp / 'plots'}/")
    return 0


if __name__ == "__main__":
    sys.exit(main())
