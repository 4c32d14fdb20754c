"""Docker id -> name mapping exporter on :9101 (reference
scripts/monitoring/docker_mapping_exporter.py:1-193).

Reads the Docker Engine API over its unix socket and exposes three all-ones gauges used by
Grafana's ``* on(interface) group_left(network_name)`` style joins:

* ``docker_network_mapping{interface="br-<id12>",network_name}`` for bridge networks;
* ``docker_container_mapping{id="/system.slice/docker-<id>.scope",container_name,
  service_name}`` (cAdvisor's ``id`` label; service = compose service label);
* ``docker_ip_mapping{ip_address,container_name,service_name}`` for addresses on
  ``INTER_AGENT_NETWORK`` (default ``infra_inter_agent_network``).

Mappings are cached for ``CACHE_TTL`` seconds (default 10).  ``DockerApi`` is injectable
so the exporter is testable without a daemon.  Label values are escaped per the
Prometheus text format.
"""
from __future__ import annotations

import http.client
import json
import os
import socket
import sys
import threading
import time
from http.server import BaseHTTPRequestHandler, HTTPServer


def _esc(v: str) -> str:
    return str(v).replace("\\", "\\\\").replace('"', '\\"').replace("\n", "\\n")


class _UnixConnection(http.client.HTTPConnection):
    def __init__(self, path: str, timeout: float = 5.0):
        super().__init__("localhost", timeout=timeout)
        self._path = path

    def connect(self):
        self.sock = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.sock.settimeout(self.timeout)
        self.sock.connect(self._path)


class DockerApi:
    def __init__(self, socket_path: str | None = None):
        self.socket_path = socket_path or os.getenv("DOCKER_SOCKET", "/var/run/docker.sock")

    def get(self, path: str):
        conn = _UnixConnection(self.socket_path)
        try:
            conn.request("GET", path)
            resp = conn.getresponse()
            body = resp.read().decode("utf-8")
        finally:
            conn.close()
        if resp.status != 200:
            print(f"Docker API error {resp.status} for {path}: {body[:200]}", file=sys.stderr)
            return None
        return json.loads(body)


def build_mappings(api, inter_agent_network: str) -> dict:
    m = {"networks": {}, "containers": {}, "ips": {}}
    for net in api.get("/networks") or []:
        nid, name = net.get("Id", ""), net.get("Name", "")
        if net.get("Driver") == "bridge" and nid and name:
            m["networks"][f"br-{nid[:12]}"] = name
    for c in api.get("/containers/json") or []:
        cid = c.get("Id", "")
        names = c.get("Names") or []
        cname = names[0].lstrip("/") if names else cid[:12]
        svc = (c.get("Labels") or {}).get("com.docker.compose.service", cname)
        m["containers"][f"/system.slice/docker-{cid}.scope"] = (cname, svc)
        nets = (c.get("NetworkSettings") or {}).get("Networks") or {}
        ip = (nets.get(inter_agent_network) or {}).get("IPAddress", "")
        if ip:
            m["ips"][ip] = (cname, svc)
    return m


class MappingExporter:
    def __init__(self, api=None, inter_agent_network: str | None = None, ttl: float | None = None):
        self.api = api or DockerApi()
        self.network = inter_agent_network or os.getenv("INTER_AGENT_NETWORK",
                                                        "infra_inter_agent_network")
        self.ttl = float(os.getenv("CACHE_TTL", "10") if ttl is None else ttl)
        self._cache = None
        self._at = 0.0
        self._lock = threading.Lock()

    def mappings(self) -> dict:
        with self._lock:
            if self._cache is not None and time.time() - self._at < self.ttl:
                return self._cache
            try:
                m = build_mappings(self.api, self.network)
            except Exception as e:  # keep serving the previous view
                print(f"Error fetching Docker mappings: {e}", file=sys.stderr, flush=True)
                m = self._cache or {"networks": {}, "containers": {}, "ips": {}}
            self._cache, self._at = m, time.time()
            return m

    def render(self) -> str:
        m = self.mappings()
        out = ["# HELP docker_network_mapping Mapping of Docker bridge interfaces to network names",
               "# TYPE docker_network_mapping gauge"]
        out += [f'docker_network_mapping{{interface="{_esc(b)}",network_name="{_esc(n)}"}} 1'
                for b, n in m["networks"].items()]
        out += ["# HELP docker_container_mapping Mapping of Docker cgroup scopes to "
                "container/service names", "# TYPE docker_container_mapping gauge"]
        out += [f'docker_container_mapping{{id="{_esc(i)}",container_name="{_esc(c)}",'
                f'service_name="{_esc(s)}"}} 1' for i, (c, s) in m["containers"].items()]
        out += ["# HELP docker_ip_mapping Mapping of Docker container IPs to names on "
                "inter_agent_network", "# TYPE docker_ip_mapping gauge"]
        out += [f'docker_ip_mapping{{ip_address="{_esc(ip)}",container_name="{_esc(c)}",'
                f'service_name="{_esc(s)}"}} 1' for ip, (c, s) in m["ips"].items()]
        return "\n".join(out) + "\n"


def make_handler(exp: MappingExporter):
    class Handler(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            if self.path != "/metrics":
                self.send_response(404)
                self.end_headers()
                return
            body = exp.render().encode()
            self.send_response(200)
            self.send_header("Content-Type", "text/plain; charset=utf-8")
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def log_message(self, *a):
            pass

    return Handler


def main() -> int:
    port = int(os.getenv("EXPORTER_PORT", "9101"))
    exp = MappingExporter()
    try:
        v = exp.api.get("/version")
        print(f"Connected to Docker {(v or {}).get('Version', '?')}", flush=True)
    except Exception as e:
        print(f"WARNING: Cannot connect to Docker: {e}", flush=True)
    print(f"Docker mapping exporter listening on port {port}", flush=True)
    HTTPServer(("0.0.0.0", port), make_handler(exp)).serve_forever()
    return 0


if __name__ == "__main__":
    sys.exit(main())
