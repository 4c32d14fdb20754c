"""Endpoint summary (reference scripts/fetch_endpoints.sh:1-338).

Turns ``docker compose ps --format json`` rows into a table of service URLs (published
ports on this host, or the distributed-mode inter-agent IPs) and prints the matching
``ssh -L`` port-forward suggestion.  ``summarize(rows)`` is pure so it is testable without
a Docker daemon.
"""
from __future__ import annotations

import argparse
import json
import subprocess
import sys

PATHS = {"llm-backend": ["/chat", "/health", "/metrics"], "agent-a": ["/task", "/agentverse"],
         "mcp-tool-db": ["/query"], "chat-ui": ["/chat/", "/agentverse/"],
         "jaeger": ["/"], "prometheus": ["/"], "grafana": ["/d/agentic-traffic-testbed"],
         "cadvisor": ["/metrics"], "docker-mapping-exporter": ["/metrics"]}


def _ports(row: dict) -> list[tuple[int, int]]:
    pubs = row.get("Publishers") or []
    out = {(p.get("PublishedPort"), p.get("TargetPort")) for p in pubs
           if isinstance(p, dict) and p.get("PublishedPort")}
    return sorted(out)


def summarize(rows: list[dict], host: str = "localhost") -> list[dict]:
    out = []
    for r in rows:
        svc = r.get("Service") or r.get("Name") or "?"
        ports = _ports(r)
        paths = PATHS.get(svc) or (["/subtask"] if svc.startswith("agent-b") else ["/"])
        urls = [f"http://{host}:{pub}{path}" for pub, _ in ports[:1] for path in paths]
        out.append({"service": svc, "state": r.get("State", "?"),
                    "ports": [p for p, _ in ports], "urls": urls})
    return sorted(out, key=lambda e: e["service"])


def compose_rows(files: list[str]) -> list[dict]:
    cmd = ["docker", "compose"]
    for f in files:
        cmd += ["-f", f]
    r = subprocess.run(cmd + ["ps", "--format", "json"], capture_output=True, text=True,
                       timeout=20)
    if r.returncode != 0:
        raise RuntimeError(r.stderr.strip() or "docker compose ps failed")
    txt = r.stdout.strip()
    if txt.startswith("["):
        return json.loads(txt)
    return [json.loads(line) for line in txt.splitlines() if line.strip().startswith("{")]


def render(entries: list[dict], ssh_target: str | None = None) -> str:
    lines = [f"{'SERVICE':<26} {'STATE':<10} URLS"]
    for e in entries:
        lines.append(f"{e['service']:<26} {e['state']:<10} {' '.join(e['urls']) or '-'}")
    ports = sorted({p for e in entries for p in e["ports"]})
    if ports:
        fwd = " ".join(f"-L {p}:localhost:{p}" for p in ports)
        lines.append("")
        lines.append(f"Port-forward from your workstation: ssh -N {fwd} "
                     f"{ssh_target or '<user>@<this-host>'}")
    return "\n".join(lines)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Print testbed service URLs")
    ap.add_argument("-f", "--file", action="append", default=[], help="compose file(s)")
    ap.add_argument("--host", default="localhost")
    ap.add_argument("--ssh-target", default=None)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args(argv)
    try:
        entries = summarize(compose_rows(a.file), a.host)
    except (OSError, RuntimeError, subprocess.SubprocessError) as e:
        print(f"[!] {e}", file=sys.stderr)
        return 1
    print(json.dumps(entries, indent=2) if a.json else render(entries, a.ssh_target))
    return 0


if __name__ == "__main__":
    sys.exit(main())
