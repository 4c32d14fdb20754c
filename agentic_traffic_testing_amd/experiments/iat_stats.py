"""Inter-arrival-time statistics (reference scripts/experiment/plot_results.py:866-1142).

``describe(vals)``: n, mean, std, CV (1 for a Poisson process), skewness, excess kurtosis,
p50/p95/p99, autocorrelation at lags 1-5 and a Ljung-Box test at lag 10.  The reference
takes Ljung-Box from statsmodels and reports NaN without it; statsmodels is not in this
image, so the statistic Q = n(n+2) sum_k r_k^2 / (n-k) and its chi-square(10) p-value are
computed here directly.

``fit(vals)``: MLE fits (location fixed at 0) of exponential, Weibull, log-normal, gamma
and Pareto with log-likelihood, AIC, BIC and a one-sample KS test, sorted by AIC.
``interpret`` / ``fit_table`` render the plain-text report lines.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import stats as st

CANDIDATES = (("expon", "Exponential (Poisson process)"), ("weibull_min", "Weibull"),
              ("lognorm", "Log-normal"), ("gamma", "Gamma"), ("pareto", "Pareto (heavy-tail)"))


def autocorr(vals: np.ndarray, lag: int) -> float:
    x = np.asarray(vals, dtype=np.float64)
    if len(x) <= lag + 1:
        return float("nan")
    a, b = x[:-lag], x[lag:]
    if a.std() == 0 or b.std() == 0:
        return float("nan")
    return float(np.corrcoef(a, b)[0, 1])


def ljung_box(vals: np.ndarray, lags: int = 10) -> tuple[float, float]:
    x = np.asarray(vals, dtype=np.float64)
    n = len(x)
    if n <= lags + 1:
        return float("nan"), float("nan")
    d = x - x.mean()
    denom = float(np.dot(d, d))
    if denom == 0:
        return float("nan"), float("nan")
    q = 0.0
    for k in range(1, lags + 1):
        rk = float(np.dot(d[:-k], d[k:])) / denom
        q += rk * rk / (n - k)
    q *= n * (n + 2)
    return q, float(st.chi2.sf(q, lags))


def describe(vals) -> dict:
    v = np.asarray(vals, dtype=np.float64)
    mean, std = float(v.mean()), float(v.std())
    lb, lbp = ljung_box(v, 10)
    return {"n": int(len(v)), "mean": mean, "std": std,
            "cv": std / mean if mean > 0 else float("nan"),
            "skewness": float(st.skew(v)) if len(v) > 2 else float("nan"),
            "kurtosis": float(st.kurtosis(v)) if len(v) > 3 else float("nan"),
            "p50": float(np.percentile(v, 50)), "p95": float(np.percentile(v, 95)),
            "p99": float(np.percentile(v, 99)),
            "acf": [autocorr(v, k) for k in range(1, 6)], "lb_stat": lb, "lb_p": lbp}


def fit(vals) -> list[dict]:
    v = np.asarray(vals, dtype=np.float64)
    v = v[v > 0]
    n = len(v)
    out = []
    if n < 3:
        return out
    for name, label in CANDIDATES:
        dist = getattr(st, name)
        try:
            params = dist.fit(v, floc=0)
            ll = float(np.sum(dist.logpdf(v, *params)))
            if not math.isfinite(ll):
                continue
            k = len(params) - 1  # location is fixed, not estimated
            ks, ksp = st.kstest(v, name, args=params)
            out.append({"name": name, "label": label, "params": tuple(map(float, params)),
                        "log_ll": ll, "aic": 2 * k - 2 * ll, "bic": k * math.log(n) - 2 * ll,
                        "ks_stat": float(ks), "ks_p": float(ksp)})
        except Exception:  # noqa: BLE001 - a failed fit is just not a candidate
            continue
    out.sort(key=lambda r: r["aic"])
    return out


def interpret(d: dict, fits: list[dict]) -> list[str]:
    lines = []
    cv = d["cv"]
    if cv < 0.8:
        lines.append(f"  CV={cv:.3f} < 1  -> more regular than Poisson")
    elif cv > 1.2:
        lines.append(f"  CV={cv:.3f} > 1  -> burstier than Poisson")
    else:
        lines.append(f"  CV={cv:.3f} ~ 1  -> variability consistent with Poisson/exponential")
    if not math.isnan(d["lb_p"]):
        if d["lb_p"] < 0.05:
            lines.append(f"  Ljung-Box p={d['lb_p']:.4f} < 0.05  -> significant autocorrelation; "
                         "arrivals are NOT independent (not pure Poisson)")
        else:
            lines.append(f"  Ljung-Box p={d['lb_p']:.4f} >= 0.05  -> independence not rejected")
    if fits:
        b = fits[0]
        lines.append(f"  Best-fit by AIC: {b['label']}  (AIC={b['aic']:.1f}, KS p={b['ks_p']:.4f})")
        lines.append(f"  KS test does NOT reject {b['label']} at alpha=0.05" if b["ks_p"] >= 0.05
                     else f"  KS test REJECTS {b['label']} at alpha=0.05 - consider a mixture "
                          "or empirical model")
    return lines


def fit_table(fits: list[dict]) -> list[str]:
    lines = [f"  {'Distribution':<36} {'AIC':>10} {'BIC':>10} {'KS stat':>9} {'KS p':>8}  "
             f"{'not rejected?':>14}", "  " + "-" * 92]
    for r in fits:
        ok = "yes (a=0.05)" if r["ks_p"] >= 0.05 else "NO"
        lines.append(f"  {r['label']:<36} {r['aic']:>10.1f} {r['bic']:>10.1f} "
                     f"{r['ks_stat']:>9.4f} {r['ks_p']:>8.4f}  {ok:>14}")
    return lines


def report(name: str, vals) -> list[str]:
    d = describe(vals)
    fits = fit(vals)
    lines = [f"== {name} ==",
             f"  n={d['n']}  mean={d['mean']:.4f}s  std={d['std']:.4f}s  cv={d['cv']:.3f}",
             f"  p50={d['p50']:.4f}s  p95={d['p95']:.4f}s  p99={d['p99']:.4f}s  "
             f"skew={d['skewness']:.3f}  kurt={d['kurtosis']:.3f}",
             "  acf(1..5)=" + ", ".join(f"{a:.3f}" for a in d["acf"]),
             f"  Ljung-Box(10): Q={d['lb_stat']:.3f}  p={d['lb_p']:.4f}"]
    if fits:
        lines += fit_table(fits)
    lines += interpret(d, fits)
    return lines
