"""Testbed health check (reference scripts/monitoring/health_check.py:1-491).

Checks, in order: compose services (running state), the LLM backend (DNS + a functional
``POST {"prompt": "test"}``), every Agent A ``/task`` and Agent B ``/subtask`` endpoint and
then the agent -> LLM critical path through each, the UI (warning only), and the
monitoring exporters (cAdvisor needs ``container_cpu_usage_seconds_total`` /
``container_memory_usage_bytes``; the TCP collector needs ``tcp_bytes_total`` /
``tcp_packets_total``; warnings only).  Exit status 0 when every critical check passed,
1 otherwise.

Differences from the reference:

* compose files are selectable (``--compose-file``, repeatable) so the distributed
  topology can be checked too (the reference only reads ``docker-compose.yml``, SURVEY
  Appendix B item 11); ``--docker-compose-dir`` still picks ``<dir>/docker-compose.yml``;
* the LLM check also reads ``GET /health`` of the backend (503 = engine stalled);
* ``--json`` prints a machine-readable report (one object per check).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
from dataclasses import asdict, dataclass
from urllib.parse import urlparse, urlunparse

import httpx

GREEN, RED, YELLOW, BLUE, RESET, BOLD = ("\033[92m", "\033[91m", "\033[93m", "\033[94m",
                                         "\033[0m", "\033[1m")
LOCAL_HOSTS = ("localhost", "127.0.0.1", "0.0.0.0")


@dataclass
class Check:
    section: str
    name: str
    ok: bool
    detail: str = ""
    critical: bool = True


class Report:
    def __init__(self, quiet: bool = False):
        self.checks: list[Check] = []
        self.quiet = quiet
        self._section = ""

    def section(self, title: str):
        self._section = title
        if not self.quiet:
            bar = "=" * 60
            print(f"\n{BOLD}{BLUE}{bar}\n{title}\n{bar}{RESET}\n")

    def add(self, name: str, ok: bool, detail: str = "", critical: bool = True) -> bool:
        self.checks.append(Check(self._section, name, ok, detail, critical))
        if not self.quiet:
            mark = f"{GREEN}✓{RESET}" if ok else (f"{RED}✗{RESET}" if critical
                                                   else f"{YELLOW}⚠{RESET}")
            print(f"{mark} {name}{' ' + detail if detail else ''}")
        return ok

    @property
    def passed(self) -> bool:
        return all(c.ok for c in self.checks if c.critical)


def resolve(host: str) -> tuple[bool, str | None]:
    try:
        return True, socket.gethostbyname(host)
    except OSError:
        return False, None


def http_check(url: str, method: str = "GET", payload: dict | None = None,
               timeout: float = 30.0) -> tuple[bool, str | None]:
    try:
        if method == "POST":
            r = httpx.post(url, json=payload, timeout=timeout, follow_redirects=True)
        else:
            r = httpx.get(url, timeout=timeout, follow_redirects=True)
    except httpx.ConnectError as e:
        return False, f"Connection error: {e}"
    except httpx.TimeoutException:
        return False, "Request timed out"
    except Exception as e:  # noqa: BLE001 - report anything as a failed check
        return False, f"Error: {e}"
    if r.is_success or r.is_redirect:
        return True, None
    return False, f"HTTP {r.status_code}: {r.text[:200]}"


def metrics_check(url: str, required: list[str], timeout: float = 5.0) -> tuple[bool, str | None]:
    try:
        r = httpx.get(url, timeout=timeout)
    except Exception as e:  # noqa: BLE001
        return False, f"Error: {e}"
    if not r.is_success:
        return False, f"HTTP {r.status_code}"
    missing = [s for s in required if s not in r.text]
    return (False, f"Missing expected metrics: {', '.join(missing)}") if missing else (True, None)


def dns_detail(url: str) -> tuple[bool, str]:
    host = urlparse(url).hostname
    if not host or host in LOCAL_HOSTS:
        return True, ""
    ok, ip = resolve(host)
    return ok, (f"{host} -> {ip}" if ok else f"DNS resolution failed for {host}")


def critical_path(agent_url: str, field: str, timeout: float = 60.0) -> tuple[bool, str | None]:
    """A real request through the agent, which must itself reach the LLM."""
    try:
        r = httpx.post(agent_url, json={field: "Say hello"}, timeout=timeout)
    except httpx.ConnectError as e:
        return False, f"Cannot connect to agent: {e}"
    except httpx.TimeoutException:
        return False, "Request to agent timed out"
    if r.status_code == 502:
        low = r.text.lower()
        if "name resolution" in low or "temporary failure" in low:
            return False, f"Agent cannot resolve LLM hostname. Error: {r.text[:200]}"
        return False, f"LLM call failed (502). Error: {r.text[:200]}"
    if r.status_code >= 500:
        return False, f"Server error: HTTP {r.status_code}: {r.text[:200]}"
    return (True, None) if r.is_success else (False, f"Unexpected status: HTTP {r.status_code}")


def compose_ps(files: list[str]) -> list[dict]:
    cmd = ["docker", "compose"]
    for f in files:
        cmd += ["-f", f]
    r = subprocess.run(cmd + ["ps", "--format", "json"], capture_output=True, text=True,
                       timeout=15)
    if r.returncode != 0:
        raise RuntimeError("docker compose not available or services not running")
    out = r.stdout.strip()
    if out.startswith("["):
        return json.loads(out)
    rows = []
    for line in out.splitlines():
        try:
            rows.append(json.loads(line))
        except json.JSONDecodeError:
            continue
    return rows


def published_ports(entry: dict) -> list[int]:
    return sorted({p["PublishedPort"] for p in entry.get("Publishers") or []
                   if isinstance(p, dict) and isinstance(p.get("PublishedPort"), int)
                   and p["PublishedPort"] > 0})


def discover_agents(rows: list[dict], default_a: list[str], default_b: list[str]):
    a, b = [], []
    for e in rows:
        svc = e.get("Service") or e.get("Name") or ""
        ports = published_ports(e)
        if svc.startswith("agent-a") and ports:
            a.append(f"http://localhost:{ports[0]}/task")
        elif svc.startswith("agent-b") and ports:
            b.append(f"http://localhost:{ports[0]}/subtask")
    return a or default_a, b or default_b


def health_url(chat_url: str) -> str:
    p = urlparse(chat_url)
    return urlunparse(p._replace(path="/health", query=""))


def run_checks(a) -> Report:
    rep = Report(quiet=a.json)
    rows = []
    files = a.compose_file or [os.path.join(a.docker_compose_dir, "docker-compose.yml")]
    if not a.skip_docker:
        rep.section("Docker Compose Services")
        existing = [f for f in files if os.path.exists(f)]
        if not existing:
            rep.add("Docker Compose file", False, f"not found: {', '.join(files)}", critical=False)
        else:
            try:
                rows = compose_ps(existing)
                state = {r.get("Service") or r.get("Name", ""): r.get("State") == "running"
                         for r in rows}
                for svc in sorted(state):
                    if svc.startswith("agent-") or svc in ("llm-backend", "chat-ui"):
                        rep.add(f"Docker service: {svc}", state[svc], f"({state[svc]})")
                for svc in ("llm-backend", "agent-a", "chat-ui"):
                    if not any(s == svc or s.startswith(svc) for s in state):
                        rep.add(f"Docker service: {svc}", False, "(not found)")
                if not any(s.startswith("agent-b") for s in state):
                    rep.add("Docker service: agent-b", False, "(not found)")
            except (OSError, RuntimeError, subprocess.SubprocessError) as e:
                rep.add("Docker Compose", False, str(e), critical=False)

    b_default = [u.strip() for u in a.agent_b_urls.split(",") if u.strip()] or [a.agent_b_url]
    a_urls, b_urls = discover_agents(rows, [a.agent_a_url], b_default)

    rep.section("LLM Server")
    dns_ok, dns = dns_detail(a.llm_url)
    llm_ok = dns_ok
    if not dns_ok:
        rep.add("LLM Server DNS", False, dns)
    else:
        ok, err = http_check(a.llm_url, "POST", {"prompt": "test", "max_tokens": 4})
        llm_ok = rep.add("LLM Server", ok, err or f"({a.llm_url}) {dns}".strip())
        hok, herr = http_check(health_url(a.llm_url), timeout=10.0)
        rep.add("LLM /health", hok, herr or "(engine loop alive)", critical=False)

    for label, urls, field in (("Agent A", a_urls, "task"), ("Agent B", b_urls, "subtask")):
        rep.section(label)
        for i, url in enumerate(urls, 1):
            name = f"{label} ({i})" if len(urls) > 1 or label == "Agent B" else label
            dok, dns = dns_detail(url)
            if not dok:
                rep.add(f"{name} endpoint", False, dns)
                continue
            ok, err = http_check(url, "POST", {field: "health check test"})
            if rep.add(f"{name} endpoint", ok, err or f"({url})") and llm_ok:
                pok, perr = critical_path(url, field)
                rep.add(f"{name} can reach LLM", pok, perr or "(successful end-to-end test)")

    rep.section("UI (Chat Console)")
    ok, err = http_check(a.ui_url, timeout=10.0)
    rep.add("UI endpoint", ok, err or f"({a.ui_url})", critical=False)

    if not a.skip_monitoring:
        rep.section("Monitoring (cAdvisor + TCP metrics)")
        ok, err = metrics_check(a.cadvisor_url, ["container_cpu_usage_seconds_total",
                                                 "container_memory_usage_bytes"])
        rep.add("cAdvisor /metrics", ok, err or f"({a.cadvisor_url})", critical=False)
        ok, err = metrics_check(a.tcp_metrics_url, ["tcp_bytes_total", "tcp_packets_total"])
        rep.add("TCP metrics collector /metrics", ok, err or f"({a.tcp_metrics_url})",
                critical=False)
    return rep


def make_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(description="Health check for the agentic traffic testbed")
    ap.add_argument("--llm-url", default=os.environ.get("LLM_SERVER_URL",
                                                        "http://localhost:8000/chat"))
    ap.add_argument("--agent-a-url", default="http://localhost:8101/task")
    ap.add_argument("--agent-b-url", default="http://localhost:8102/subtask")
    ap.add_argument("--agent-b-urls", default=os.environ.get("AGENT_B_URLS", ""),
                    help="comma-separated Agent B endpoints (overrides discovery)")
    ap.add_argument("--ui-url", default="http://localhost:3000")
    ap.add_argument("--cadvisor-url", default="http://localhost:8080/metrics")
    ap.add_argument("--tcp-metrics-url", default="http://localhost:9100/metrics")
    ap.add_argument("--docker-compose-dir", default="infra")
    ap.add_argument("--compose-file", action="append", default=None,
                    help="compose file(s) to inspect (repeatable)")
    ap.add_argument("--skip-docker", action="store_true")
    ap.add_argument("--skip-monitoring", action="store_true")
    ap.add_argument("--json", action="store_true", help="print a JSON report")
    return ap


def main(argv: list[str] | None = None) -> int:
    a = make_parser().parse_args(argv)
    rep = run_checks(a)
    if a.json:
        print(json.dumps({"passed": rep.passed, "checks": [asdict(c) for c in rep.checks]},
                         indent=2))
    else:
        rep.section("Summary")
        if rep.passed:
            print(f"{GREEN}{BOLD}✓ All critical checks passed!{RESET}")
        else:
            print(f"{RED}{BOLD}✗ Some checks failed. Please review the errors above.{RESET}")
            print(f"\n{YELLOW}Common issues:{RESET}")
            print("  1. LLM server not running or not reachable")
            print("  2. Agent containers cannot resolve the LLM hostname (check LLM_SERVER_URL)")
            print("  3. Services not started: cd infra && docker compose up -d")
            print("  4. Port conflicts on 8000 / 8101 / 8102")
    return 0 if rep.passed else 1


if __name__ == "__main__":
    sys.exit(main())
