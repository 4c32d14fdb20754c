"""Prometheus HTTP API client shared by the scraper and the correlator.

``PromClient(base_url, fetch=None)``: ``range(expr, start, end, step)`` returns
``[{"labels", "values": [(ts, v), ...]}]`` and ``instant(expr, t)`` returns
``[{"metric", "value"}]``; NaN / +-Inf samples are dropped and failed queries are warned
about on stderr and yield ``[]`` (a scrape must never abort an experiment).  ``fetch`` is
injectable (tests run against canned JSON, no server).
"""
from __future__ import annotations

import json
import sys
import urllib.error
import urllib.parse
import urllib.request

BAD = ("NaN", "+Inf", "-Inf")


def _http_get(url: str, timeout: float = 30.0) -> dict:
    try:
        with urllib.request.urlopen(url, timeout=timeout) as r:
            return json.loads(r.read().decode())
    except urllib.error.HTTPError as e:
        raise RuntimeError(f"HTTP {e.code}: {e.read().decode()[:200]}") from e
    except Exception as e:  # noqa: BLE001 - surfaced as a warning by the caller
        raise RuntimeError(str(e)) from e


class PromClient:
    def __init__(self, base_url: str = "http://localhost:9090", fetch=None, timeout: float = 30.0):
        self.base = base_url.rstrip("/")
        self.fetch = fetch or (lambda url: _http_get(url, timeout))

    def _call(self, path: str, params: dict, expr: str) -> list:
        url = f"{self.base}{path}?{urllib.parse.urlencode(params)}"
        try:
            data = self.fetch(url)
        except RuntimeError as e:
            print(f"  WARN  prometheus query failed [{expr[:70]}]: {e}", file=sys.stderr)
            return []
        if data.get("status") != "success":
            print(f"  WARN  prometheus non-success [{expr[:70]}]: {data.get('error', '')}",
                  file=sys.stderr)
            return []
        return data.get("data", {}).get("result", [])

    def range(self, expr: str, start_s: float, end_s: float, step_s: float) -> list[dict]:
        out = []
        for s in self._call("/api/v1/query_range", {"query": expr, "start": f"{start_s:.3f}",
                                                     "end": f"{end_s:.3f}", "step": str(step_s)},
                            expr):
            vals = [(float(t), float(v)) for t, v in s.get("values", []) if v not in BAD]
            if vals:
                out.append({"labels": s.get("metric", {}), "values": vals})
        return out

    def instant(self, expr: str, t: float) -> list[dict]:
        out = []
        for s in self._call("/api/v1/query", {"query": expr, "time": f"{t:.3f}"}, expr):
            tv = s.get("value")
            if tv and tv[1] not in BAD:
                out.append({"metric": s.get("metric", {}), "value": float(tv[1])})
        return out

    def scalar_sum(self, expr: str, t: float) -> float | None:
        r = self.instant(expr, t)
        return round(sum(x["value"] for x in r), 6) if r else None

    def first(self, expr: str, t: float) -> float | None:
        r = self.instant(expr, t)
        return round(r[0]["value"], 6) if r else None
