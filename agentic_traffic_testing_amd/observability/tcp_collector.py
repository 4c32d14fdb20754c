"""L2 -> L4 TCP metrics: parse ``tcpdump -l -n -tt`` lines, export ``tcp_*`` on :9100.

Metric contract of reference scripts/monitoring/tcp_metrics_collector.py:307-396 (SURVEY
§5.5.2) - names, label sets, bucket edges and the quirks the Grafana dashboard and the
correlator rely on are kept:

* ``tcp_collector_uptime_seconds`` (gauge), ``tcp_collector_packets_processed`` (counter);
* ``tcp_{packets,bytes,syn,fin,rst}_total{src_service,dst_service}`` - bytes are the
  tcpdump ``length`` field (TCP payload), SYN counts exclude SYN-ACKs;
* ``tcp_flows_active`` (gauge);
* cumulative ``*_bucket`` series typed ``counter`` with no ``_sum`` / ``_count``:
  ``tcp_packet_size_bytes_bucket{le}``, ``tcp_flow_duration_seconds_bucket{src,dst,le}``,
  ``tcp_rtt_handshake_seconds_bucket{src,dst,le}`` (SYN -> SYN-ACK by 4-tuple, labelled
  client -> server);
* services come from ``SERVICE_IPS`` (the distributed topology's inter_agent_network and
  tools_network addresses); anything else is ``external``.

Deliberate fixes, each switchable back with
``--legacy-flow-accounting``:

* a flow's duration is observed ONCE - at its first FIN, or at idle eviction if it never
  saw one (the reference observes every FIN *and* again at eviction);
* idle eviction runs on packet time (last packet timestamp + wall time since it arrived),
  so replayed captures (``--read-stdin`` from an old pcap) age out correctly.

``ensure_port_free`` in the reference kills whatever owns the port; here that is opt-in
(``--kill-port-owner``).  State lives in one ``TcpAggregator`` object (no module globals)
so tests and embedders can run several.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import signal
import subprocess
import sys
import threading
import time
from collections import defaultdict
from dataclasses import dataclass
from datetime import datetime
from http.server import BaseHTTPRequestHandler, HTTPServer

SERVICE_IPS = {
    "172.23.0.10": "agent_a",
    "172.23.0.20": "agent_b_1",
    "172.23.0.21": "agent_b_2",
    "172.23.0.22": "agent_b_3",
    "172.23.0.23": "agent_b_4",
    "172.23.0.24": "agent_b_5",
    "172.23.0.30": "llm_backend",
    "172.23.0.40": "mcp_tool_db",
    "172.23.0.50": "chat_ui",
    "172.23.0.60": "jaeger",
    "172.24.0.10": "mcp_tool_db",
}

SIZE_EDGES = (64, 128, 256, 512, 1024, 1500, 4096, 9000)
SIZE_LABELS = tuple(str(e) for e in SIZE_EDGES) + ("inf",)
DURATION_EDGES = (0.001, 0.01, 0.1, 0.5, 1.0, 5.0, 30.0, 60.0, 300.0)
DURATION_LABELS = tuple(str(e) for e in DURATION_EDGES) + ("inf",)
RTT_EDGES = (0.0005, 0.001, 0.005, 0.01, 0.05, 0.1, 0.5, 1.0, 5.0)
RTT_LABELS = tuple(str(e) for e in RTT_EDGES) + ("inf",)

_LINE = re.compile(r"(\d+\.\d+)\s+IP\s+(\d+\.\d+\.\d+\.\d+)\.(\d+)\s+>\s+"
                   r"(\d+\.\d+\.\d+\.\d+)\.(\d+):\s+Flags\s+\[([^\]]+)\].*?length\s+(\d+)")


def bucket(value: float, edges, labels) -> str:
    for e, lab in zip(edges, labels):
        if value <= e:
            return lab
    return "inf"


@dataclass
class Packet:
    ts: float
    src_ip: str
    src_port: int
    dst_ip: str
    dst_port: int
    flags: str
    length: int


def parse_line(line: str) -> Packet | None:
    """``1772100649.468003 IP 172.23.0.10.8101 > 172.23.0.30.8000: Flags [S], ..., length 0``"""
    m = _LINE.search(line)
    if not m:
        return None
    ts, sip, sport, dip, dport, flags, length = m.groups()
    return Packet(float(ts), sip, int(sport), dip, int(dport), flags, int(length))


@dataclass
class Flow:
    src_service: str
    dst_service: str
    start: float
    last: float
    packets: int = 0
    bytes: int = 0
    fin_seen: bool = False
    duration_recorded: bool = False


class TcpAggregator:
    def __init__(self, service_ips: dict | None = None, legacy: bool = False):
        self.service_ips = dict(SERVICE_IPS if service_ips is None else service_ips)
        self.legacy = legacy
        self.lock = threading.Lock()
        self.started = time.time()
        self.processed = 0
        self.packets = defaultdict(int)
        self.bytes = defaultdict(int)
        self.syn = defaultdict(int)
        self.fin = defaultdict(int)
        self.rst = defaultdict(int)
        self.size_hist = defaultdict(int)
        self.duration_hist = defaultdict(int)   # (src, dst, le) -> count
        self.rtt_hist = defaultdict(int)        # (client, server, le) -> count
        self.pending_syn: dict = {}             # (cip, cport, sip, sport) -> ts
        self.flows: dict = {}
        self._last_pkt_ts = None
        self._last_pkt_wall = 0.0

    def service(self, ip: str) -> str:
        return self.service_ips.get(ip, "external")

    def clock(self) -> float:
        """Packet-time 'now' (falls back to wall time before any packet)."""
        if self._last_pkt_ts is None:
            return time.time()
        return self._last_pkt_ts + (time.monotonic() - self._last_pkt_wall)

    # ------------------------------------------------------------------------------------
    def ingest(self, line: str) -> bool:
        pkt = parse_line(line)
        if pkt is None:
            return False
        self.process(pkt)
        return True

    def process(self, p: Packet) -> None:
        s_src, s_dst = self.service(p.src_ip), self.service(p.dst_ip)
        pair = (s_src, s_dst)
        key = tuple(sorted(((p.src_ip, p.src_port), (p.dst_ip, p.dst_port))))
        syn, ack = "S" in p.flags, "." in p.flags
        with self.lock:
            if self._last_pkt_ts is None or p.ts >= self._last_pkt_ts:
                self._last_pkt_ts, self._last_pkt_wall = p.ts, time.monotonic()
            self.processed += 1
            self.packets[pair] += 1
            self.bytes[pair] += p.length
            self.size_hist[bucket(p.length, SIZE_EDGES, SIZE_LABELS)] += 1
            if syn and not ack:
                self.syn[pair] += 1
                self.pending_syn[(p.src_ip, p.src_port, p.dst_ip, p.dst_port)] = p.ts
            elif syn and ack:
                t0 = self.pending_syn.pop((p.dst_ip, p.dst_port, p.src_ip, p.src_port), None)
                if t0 is not None:
                    le = bucket(p.ts - t0, RTT_EDGES, RTT_LABELS)
                    self.rtt_hist[(s_dst, s_src, le)] += 1  # client -> server
            if "F" in p.flags:
                self.fin[pair] += 1
            if "R" in p.flags:
                self.rst[pair] += 1
            fl = self.flows.get(key)
            if fl is None:
                fl = self.flows[key] = Flow(s_src, s_dst, p.ts, p.ts)
            fl.last = p.ts
            fl.packets += 1
            fl.bytes += p.length
            if "F" in p.flags:
                fl.fin_seen = True
                if self.legacy or not fl.duration_recorded:
                    self._observe_duration(fl, p.ts - fl.start)

    def _observe_duration(self, fl: Flow, d: float):
        fl.duration_recorded = True
        self.duration_hist[(fl.src_service, fl.dst_service,
                            bucket(d, DURATION_EDGES, DURATION_LABELS))] += 1

    def sweep(self, max_idle: float = 60.0, now: float | None = None) -> int:
        """Evict flows idle for ``max_idle`` seconds (packet time); returns the count."""
        with self.lock:
            now = self.clock() if now is None else now
            dead = [k for k, f in self.flows.items() if now - f.last > max_idle]
            for k in dead:
                f = self.flows.pop(k)
                if self.legacy or not f.duration_recorded:
                    self._observe_duration(f, f.last - f.start)
            # SYNs never answered within the idle window will never be
            stale = [k for k, t in self.pending_syn.items() if now - t > max_idle]
            for k in stale:
                del self.pending_syn[k]
            return len(dead)

    # ------------------------------------------------------------------------------------
    def render(self) -> str:
        out = []

        def head(name, help_, typ):
            out.append(f"# HELP {name} {help_}")
            out.append(f"# TYPE {name} {typ}")

        def pairs(name, help_, d):
            head(name, help_, "counter")
            for (a, b), v in d.items():
                out.append(f'{name}{{src_service="{a}",dst_service="{b}"}} {v}')

        def hist(name, help_, d, labels):
            head(name, help_, "counter")
            for a, b in sorted({(a, b) for a, b, _ in d}):
                run = 0
                for lab in labels:
                    run += d.get((a, b, lab), 0)
                    out.append(f'{name}{{src_service="{a}",dst_service="{b}",le="{lab}"}} {run}')

        with self.lock:
            head("tcp_collector_uptime_seconds", "Time since collector started", "gauge")
            out.append(f"tcp_collector_uptime_seconds {time.time() - self.started:.2f}")
            head("tcp_collector_packets_processed", "Total packets processed", "counter")
            out.append(f"tcp_collector_packets_processed {self.processed}")
            pairs("tcp_packets_total", "Total TCP packets", self.packets)
            pairs("tcp_bytes_total", "Total TCP bytes", self.bytes)
            pairs("tcp_syn_total", "TCP SYN packets (new connections)", self.syn)
            pairs("tcp_fin_total", "TCP FIN packets (closed connections)", self.fin)
            pairs("tcp_rst_total", "TCP RST packets (reset connections)", self.rst)
            head("tcp_flows_active", "Currently active TCP flows", "gauge")
            out.append(f"tcp_flows_active {len(self.flows)}")
            head("tcp_packet_size_bytes_bucket", "TCP packet size distribution", "counter")
            run = 0
            for lab in SIZE_LABELS:
                run += self.size_hist.get(lab, 0)
                out.append(f'tcp_packet_size_bytes_bucket{{le="{lab}"}} {run}')
            hist("tcp_flow_duration_seconds_bucket",
                 "TCP flow duration distribution by service pair", self.duration_hist,
                 DURATION_LABELS)
            hist("tcp_rtt_handshake_seconds_bucket",
                 "TCP SYN/SYN-ACK RTT distribution by service pair", self.rtt_hist, RTT_LABELS)
        return "\n".join(out) + "\n"


# ---- HTTP + capture plumbing -------------------------------------------------------------
def make_handler(agg: TcpAggregator):
    class Handler(BaseHTTPRequestHandler):
        def do_GET(self):  # noqa: N802
            if self.path == "/metrics":
                body = agg.render().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; charset=utf-8")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)
            elif self.path == "/health":
                self.send_response(200)
                self.send_header("Content-Type", "text/plain")
                self.end_headers()
                self.wfile.write(b"OK")
            else:
                self.send_response(404)
                self.end_headers()

        def log_message(self, *a):
            pass

    return Handler


def log(msg: str) -> None:
    print(f"[{datetime.now().strftime('%Y-%m-%d %H:%M:%S')}] {msg}", flush=True)


def find_docker_bridge(name_filter: str = "inter_agent") -> str | None:
    """``br-<first 12 of the network id>`` of the inter-agent bridge, if it exists."""
    try:
        r = subprocess.run(["docker", "network", "ls", "--filter", f"name={name_filter}",
                            "--format", "{{.ID}}"], capture_output=True, text=True, timeout=10)
        nid = r.stdout.strip().splitlines()[0] if r.stdout.strip() else ""
        if nid:
            br = f"br-{nid[:12]}"
            if subprocess.run(["ip", "link", "show", br], capture_output=True).returncode == 0:
                return br
    except (OSError, subprocess.SubprocessError):
        pass
    return None


def port_owner_pids(port: int) -> list[int]:
    try:
        r = subprocess.run(["lsof", "-ti", f":{port}"], capture_output=True, text=True, timeout=5)
        return [int(x) for x in r.stdout.split()]
    except (OSError, subprocess.SubprocessError, ValueError):
        return []


def load_service_ips(spec: str | None) -> dict:
    """``--service-ips`` / ``TCP_SERVICE_IPS``: JSON object or path to a JSON file."""
    spec = spec or os.environ.get("TCP_SERVICE_IPS")
    if not spec:
        return dict(SERVICE_IPS)
    text = open(spec).read() if os.path.exists(spec) else spec
    return {str(k): str(v) for k, v in json.loads(text).items()}


def feed(agg: TcpAggregator, stream) -> None:
    for line in stream:
        agg.ingest(line)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Collect TCP metrics and expose them to Prometheus")
    ap.add_argument("--interface", "-i", help="capture interface (default: inter-agent bridge)")
    ap.add_argument("--filter", "-f", default="tcp and net 172.23.0.0/24")
    ap.add_argument("--port", "-p", type=int, default=9100)
    ap.add_argument("--cleanup-interval", type=int, default=30)
    ap.add_argument("--max-idle", type=float, default=60.0, help="flow idle eviction (s)")
    ap.add_argument("--sudo-tcpdump", action="store_true")
    ap.add_argument("--read-stdin", action="store_true",
                    help="read tcpdump -l -n -tt lines from stdin (sudo tcpdump ... | collector)")
    ap.add_argument("--service-ips", default=None, help="JSON map or file: ip -> service")
    ap.add_argument("--legacy-flow-accounting", action="store_true",
                    help="reference behaviour: flow duration at every FIN and at eviction")
    ap.add_argument("--kill-port-owner", action="store_true",
                    help="SIGTERM whatever listens on --port first (reference behaviour)")
    a = ap.parse_args(argv)

    agg = TcpAggregator(load_service_ips(a.service_ips), legacy=a.legacy_flow_accounting)
    if a.kill_port_owner:
        for pid in port_owner_pids(a.port):
            log(f"[*] Killing process {pid} using port {a.port}")
            try:
                os.kill(pid, signal.SIGTERM)
            except OSError as e:
                log(f"[!] Could not kill PID {pid}: {e}")
        time.sleep(1)
    srv = HTTPServer(("0.0.0.0", a.port), make_handler(agg))
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    log(f"[*] Metrics endpoint: http://localhost:{a.port}/metrics")

    def sweeper():
        while True:
            time.sleep(a.cleanup_interval)
            agg.sweep(a.max_idle)

    threading.Thread(target=sweeper, daemon=True).start()

    def stop(signum, frame):
        log("[*] Shutting down...")
        srv.shutdown()
        sys.exit(0)

    signal.signal(signal.SIGINT, stop)
    signal.signal(signal.SIGTERM, stop)
    if a.read_stdin:
        log("[*] Reading tcpdump lines from stdin")
        feed(agg, sys.stdin)
        return 0
    iface = a.interface or find_docker_bridge() or "any"
    cmd = ["tcpdump", "-i", iface, "-l", "-n", "-tt", a.filter]
    if a.sudo_tcpdump:
        cmd = ["sudo"] + cmd
    log(f"[*] Starting tcpdump: {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                            bufsize=1)
    try:
        feed(agg, proc.stdout)
    finally:
        proc.terminate()
    return 0


if __name__ == "__main__":
    sys.exit(main())
