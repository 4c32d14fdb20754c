"""Grafana dashboard + Prometheus / Grafana provisioning generator.

The reference checks in a 3,112-line hand-edited dashboard JSON
(infra/monitoring/grafana/provisioning/dashboards/agentic-traffic.json).  Its panel
*titles* and *PromQL* are a contract: the experiment scraper walks the dashboard for its
query list and the plotter keys on titles.  Here the dashboard is a
declarative spec - rows of panels, each with title, unit and (expr, legend) targets - and
the JSON is generated (``python -m agentic_traffic_testing_amd.observability.dashboard``
rewrites ``infra/monitoring/grafana/provisioning/dashboards/agentic-traffic.json``).

Contract kept: dashboard uid ``agentic-traffic-testbed``, title "Agentic Traffic Testbed",
5 s refresh, datasource template variable, the 8 reference rows in order with their panel
titles and expressions.  Fixed: panel ids are unique (the reference duplicates id 301,
Appendix B item 11) and each panel sits inside its own row in grid order (the reference
places "LLM Interarrival Time" geometrically under the Interarrival row although it is
listed with AI Performance).  Added: a ninth row, "MI355X Engine", for this backend's
engine gauges (step time, running / waiting sequences, KV free blocks, prefix-cache hit
rate, fine-bucket TTFT ``llm_ttft_seconds``) - the contract histogram's lowest TTFT bucket
is 0.5 s, too coarse for this hardware.
"""
from __future__ import annotations

import argparse
import json
from dataclasses import dataclass, field
from pathlib import Path

UID = "agentic-traffic-testbed"
TITLE = "Agentic Traffic Testbed"
DS = {"type": "prometheus", "uid": "${datasource}"}


@dataclass
class Panel:
    title: str
    targets: list                 # [(expr, legend | None)]
    unit: str = "short"
    kind: str = "timeseries"      # timeseries | stat
    w: int = 12
    h: int = 8
    description: str = ""


@dataclass
class Row:
    title: str
    panels: list = field(default_factory=list)


def _q(p: float, metric: str, sel: str = "", window: str = "5m") -> str:
    return (f"histogram_quantile({p}, sum by (le) (rate({metric}_bucket{sel}[{window}])))")


_CADV_DOCKER = 'id=~"/system.slice/docker-.*\\\\.scope"'
_BR = 'id="/",interface=~"br-.*"'
_JOIN_NET = " * on(interface) group_left(network_name) docker_network_mapping"
_A_LLM = '{src_service="agent_a",dst_service="llm_backend"}'
_BURST = "max_over_time(rate(llm_requests_total[10s])[5m:10s])"


def _p50_p95(metric: str, what: str, unit: str = "s", w: int = 12, sel: str = "") -> list:
    return [(_q(0.5, metric, sel), f"p50 [5m] {what}"), (_q(0.95, metric, sel), f"p95 [5m] {what}")]


def spec() -> list[Row]:
    rate_sv = [('rate(llm_requests_total{status="success"}[30s])', "success req/s"),
               ('rate(llm_requests_total{status="error"}[30s])', "error req/s")]
    return [
        Row("Overview", [
            Panel("Active Containers (Docker)",
                  [(f'count(container_cpu_usage_seconds_total{{cpu="total",{_CADV_DOCKER}}})', None)],
                  w=6, h=6),
            Panel("Docker Network TX Rate",
                  [(f"sum(rate(container_network_transmit_bytes_total{{{_BR}}}[1m]))", None)],
                  unit="Bps", w=6, h=6),
            Panel("Docker Network RX Rate",
                  [(f"sum(rate(container_network_receive_bytes_total{{{_BR}}}[1m]))", None)],
                  unit="Bps", w=6, h=6),
            Panel("LLM Request Rate — success vs error", rate_sv, w=18),
        ]),
        Row("Network Traffic", [
            Panel("Network Transmit Rate by Interface",
                  [(f"rate(container_network_transmit_bytes_total{{{_BR}}}[30s]){_JOIN_NET}",
                    "{{network_name}} TX")], unit="Bps"),
            Panel("Network Receive Rate by Interface",
                  [(f"rate(container_network_receive_bytes_total{{{_BR}}}[30s]){_JOIN_NET}",
                    "{{network_name}} RX")], unit="Bps"),
            Panel("Packets Transmitted (by Interface)",
                  [(f"rate(container_network_transmit_packets_total{{{_BR}}}[30s]){_JOIN_NET}",
                    "{{network_name}}")], unit="pps"),
            Panel("Packets per Minute (by Interface)",
                  [(f"increase(container_network_transmit_packets_total{{{_BR}}}[1m]){_JOIN_NET}",
                    "{{network_name}}")]),
        ]),
        Row("Resource Usage", [
            Panel("CPU (core equivalents per container)",
                  [("sum by (id) (rate(container_cpu_usage_seconds_total{cpu=\"total\","
                    f"{_CADV_DOCKER}}}[1m])) * on(id) group_left(service_name) "
                    "docker_container_mapping", "{{service_name}}")]),
            Panel("Memory Usage per container",
                  [(f"container_memory_usage_bytes{{{_CADV_DOCKER}}} * on(id) "
                    "group_left(service_name) docker_container_mapping", "{{service_name}}")],
                  unit="bytes"),
        ]),
        Row("Service-level Network (TCP)", [
            Panel("TCP Bytes/s by Service Pair",
                  [('rate(tcp_bytes_total{src_service!="external",dst_service!="external",'
                    'src_service!="jaeger",dst_service!="jaeger"}[1m])',
                    "{{src_service}} → {{dst_service}}")], unit="Bps"),
            Panel("TCP Bytes/s from LLM Backend",
                  [('sum(rate(tcp_bytes_total{src_service="llm_backend",'
                    'dst_service!="external"}[1m]))', "from llm_backend")], unit="Bps"),
            Panel("TCP RTT (SYN/SYN-ACK Agent A → LLM)",
                  _p50_p95("tcp_rtt_handshake_seconds", "RTT AgentA → LLM", sel=_A_LLM),
                  unit="s"),
            Panel("TCP Flow Duration (Agent A → LLM)",
                  _p50_p95("tcp_flow_duration_seconds", "AgentA → LLM", sel=_A_LLM), unit="s"),
        ]),
        Row("AI Performance (LLM)", [
            Panel("LLM End-to-end Latency (p50/p95)",
                  _p50_p95("llm_request_latency_seconds", "latency"), unit="s"),
            Panel("LLM Time-to-First-Token (TTFT p50/p95)",
                  _p50_p95("llm_queue_wait_seconds", "TTFT"), unit="s"),
            Panel("Prompt Tokens / s", [("rate(llm_prompt_tokens_total[1m])", "prompt tokens/s")],
                  w=8, h=6),
            Panel("Completion Tokens / s",
                  [("rate(llm_completion_tokens_total[1m])", "completion tokens/s")], w=8, h=6),
            Panel("In-flight LLM Requests", [("llm_inflight_requests", "in-flight requests")],
                  w=8, h=6),
            Panel("LLM Tokens & In-flight Requests (overlay)",
                  [("rate(llm_prompt_tokens_total[1m])", "prompt tokens/s"),
                   ("rate(llm_completion_tokens_total[1m])", "completion tokens/s"),
                   ("llm_inflight_requests", "in-flight requests")], w=24, h=6),
        ]),
        Row("LLM Configuration", [
            Panel("KV-cache-limited max concurrency",
                  [("llm_kv_cache_est_max_concurrency_at_max_model_len",
                    "KV-cache-limited max concurrency")], kind="stat", w=6, h=4),
            Panel("vLLM max_num_batched_tokens",
                  [("llm_config_max_num_batched_tokens", "max_num_batched_tokens")],
                  kind="stat", w=6, h=4),
            Panel("Max tokens per generation (LLM_MAX_TOKENS)",
                  [("llm_config_max_tokens", "max_tokens")], kind="stat", w=6, h=4),
            Panel("GPU memory utilization target",
                  [("llm_config_gpu_memory_utilization", "gpu_memory_utilization")],
                  unit="percentunit", kind="stat", w=6, h=4),
            Panel("LLM Errors — total (since restart)",
                  [('llm_requests_total{status="error"}', "LLM errors")], kind="stat", w=6, h=4),
            Panel("LLM Errors — last 1 h",
                  [('increase(llm_requests_total{status="error"}[1h])', "errors last 1h")],
                  kind="stat", w=6, h=4),
            Panel("Free Concurrent Slots (KV-cache capacity − in-flight)",
                  [("clamp_min(llm_computed_max_concurrency - llm_inflight_requests, 0)",
                    "Free concurrent slots"),
                   ("llm_computed_max_concurrency", "Max concurrency (KV-cache)")],
                  kind="stat", w=12, h=4),
        ]),
        Row("Interarrival Interpretation", [
            Panel("LLM Interarrival Time (30s rolling avg)",
                  [("1 / sum(rate(llm_requests_total[30s]))", "avg interarrival (s)")], unit="s"),
            Panel("Request arrivals in last 4s (by status)",
                  [('increase(llm_requests_total{status="success"}[4s])',
                    "success (arrivals in last 4s)"),
                   ('increase(llm_requests_total{status="error"}[4s])',
                    "error (arrivals in last 4s)")]),
            Panel("LLM Request Rate — success vs error (30s window)", rate_sv, w=8),
            Panel("LLM End-to-end Latency (p50/p95)",
                  _p50_p95("llm_request_latency_seconds", "latency"), unit="s", w=8),
            Panel("LLM Time-to-First-Token (TTFT p50/p95)",
                  _p50_p95("llm_queue_wait_seconds", "TTFT"), unit="s", w=8),
            Panel("Concurrent In-flight Requests (burst signature)",
                  [("llm_inflight_requests", "in-flight requests")], w=24, h=6),
        ]),
        Row("Traffic Characterization", [
            Panel("Interarrival Jitter (p95 − p50)",
                  _p50_p95("llm_interarrival_seconds", "interarrival")
                  + [(f"{_q(0.95, 'llm_interarrival_seconds')} - "
                      f"{_q(0.5, 'llm_interarrival_seconds')}", "jitter p95-p50 [5m]")],
                  unit="s", w=8),
            Panel("Queue Wait Distribution (p50/p95/p99) + In-flight",
                  _p50_p95("llm_queue_wait_seconds", "queue wait")
                  + [(_q(0.99, "llm_queue_wait_seconds"), "p99 [5m] queue wait"),
                     ("llm_inflight_requests", "in-flight (queue proxy)")], unit="s", w=8),
            Panel("Burstiness Coefficient (peak 10s / avg 5m)",
                  [(f"{_BURST} / rate(llm_requests_total[5m])",
                    "burstiness (peak 10s / avg 5m)"),
                   ("rate(llm_requests_total[5m])", "avg throughput (req/s)"),
                   (_BURST, "peak 10s throughput (req/s)")], w=8),
        ]),
        Row("MI355X Engine", [
            Panel("Engine Step Time (p50/p95)", _p50_p95("llm_engine_step_seconds", "step"),
                  unit="s", w=8),
            Panel("TTFT fine buckets (p50/p95/p99)",
                  _p50_p95("llm_ttft_seconds", "TTFT")
                  + [(_q(0.99, "llm_ttft_seconds"), "p99 [5m] TTFT")], unit="s", w=8),
            Panel("Engine Steps / s", [("rate(llm_engine_steps_total[1m])", "steps/s")], w=8),
            Panel("Running / Waiting Sequences",
                  [("llm_engine_running_sequences", "running"),
                   ("llm_engine_waiting_sequences", "waiting")], w=8),
            Panel("KV Cache Free Blocks",
                  [("llm_kv_cache_free_blocks", "free blocks"),
                   ("llm_kv_cache_num_gpu_blocks", "total blocks")], w=8),
            Panel("Prefix-cache Hit Rate",
                  [("llm_prefix_cache_hit_blocks / clamp_min(llm_prefix_cache_query_blocks, 1)",
                    "hit rate")], unit="percentunit", w=8),
            Panel("Engine Heartbeat Age", [("llm_engine_heartbeat_age_seconds", "heartbeat age")],
                  unit="s", w=24, h=5),
        ]),
    ]


def _panel_json(p: Panel, pid: int, x: int, y: int) -> dict:
    targets = []
    for i, (expr, legend) in enumerate(p.targets):
        t = {"datasource": DS, "expr": expr, "refId": chr(ord("A") + i)}
        if legend:
            t["legendFormat"] = legend
        targets.append(t)
    d = {"id": pid, "type": p.kind, "title": p.title, "datasource": DS,
         "gridPos": {"h": p.h, "w": p.w, "x": x, "y": y}, "targets": targets,
         "fieldConfig": {"defaults": {"unit": p.unit}, "overrides": []}}
    if p.description:
        d["description"] = p.description
    if p.kind == "stat":
        d["options"] = {"reduceOptions": {"calcs": ["lastNotNull"], "fields": "",
                                          "values": False}, "colorMode": "value",
                        "graphMode": "area", "textMode": "auto"}
    else:
        d["options"] = {"legend": {"displayMode": "list", "placement": "bottom",
                                   "showLegend": True},
                        "tooltip": {"mode": "multi", "sort": "none"}}
        d["fieldConfig"]["defaults"]["custom"] = {"drawStyle": "line", "lineWidth": 1,
                                                  "fillOpacity": 10, "showPoints": "never"}
    return d


def build_dashboard(rows: list[Row] | None = None) -> dict:
    rows = spec() if rows is None else rows
    panels, y, pid = [], 0, 1
    for ri, row in enumerate(rows):
        panels.append({"id": 1000 + ri, "type": "row", "title": row.title, "collapsed": False,
                       "gridPos": {"h": 1, "w": 24, "x": 0, "y": y}, "panels": []})
        y += 1
        x, line_h = 0, 0
        for p in row.panels:
            if x + p.w > 24:
                y, x, line_h = y + line_h, 0, 0
            panels.append(_panel_json(p, pid, x, y))
            pid += 1
            x += p.w
            line_h = max(line_h, p.h)
        y += line_h
    return {
        "annotations": {"list": []}, "editable": True, "fiscalYearStartMonth": 0,
        "graphTooltip": 1, "id": None, "links": [], "liveNow": False, "panels": panels,
        "refresh": "5s", "schemaVersion": 38, "style": "dark",
        "tags": ["agentic", "traffic", "testbed", "mi355x"],
        "templating": {"list": [{"current": {"selected": False, "text": "Prometheus",
                                             "value": "Prometheus"},
                                 "hide": 0, "includeAll": False, "label": "Datasource",
                                 "multi": False, "name": "datasource", "options": [],
                                 "query": "prometheus", "refresh": 1, "regex": "",
                                 "skipUrlSync": False, "type": "datasource"}]},
        "time": {"from": "now-15m", "to": "now"}, "timepicker": {}, "timezone": "",
        "title": TITLE, "uid": UID, "version": 1, "weekStart": "",
    }


# ---- Prometheus + Grafana provisioning ----------------------------------------------------
def prometheus_config(mode: str = "single") -> str:
    """prometheus.yml (reference infra/monitoring/prometheus.yml:1-76).  Fixed: the agent
    jobs are dropped - agents expose no /metrics (Appendix B item 5)."""
    llm = "llm-backend:8000" if mode == "single" else "172.23.0.30:8000"
    return f"""# Generated by agentic_traffic_testing_amd.observability.dashboard - edit the spec there.
global:
  scrape_interval: 5s
  evaluation_interval: 5s

scrape_configs:
  - job_name: prometheus
    static_configs:
      - targets: ["localhost:9090"]

  # host-mode cAdvisor: container_* and bridge-level (id="/") network series
  - job_name: cadvisor
    static_configs:
      - targets: ["host.docker.internal:8080"]
    relabel_configs:
      - source_labels: [__address__]
        regex: "host.docker.internal:8080"
        target_label: __address__
        replacement: "172.17.0.1:8080"

  # tcp_* from scripts/monitoring/run_tcpdump.sh (host, :9100)
  - job_name: tcp-metrics
    static_configs:
      - targets: ["172.17.0.1:9100"]
        labels:
          source: tcpdump

  # llm_* from the MI355X backend
  - job_name: llm-backend
    scrape_interval: 2s
    metrics_path: /metrics
    static_configs:
      - targets: ["{llm}"]

  # docker_*_mapping join helpers
  - job_name: docker-mapping
    scrape_interval: 10s
    static_configs:
      - targets: ["docker-mapping-exporter:9101"]
"""


DATASOURCES_YML = """# Generated by agentic_traffic_testing_amd.observability.dashboard
apiVersion: 1
datasources:
  - name: Prometheus
    type: prometheus
    uid: prometheus
    access: proxy
    url: http://prometheus:9090
    isDefault: true
    jsonData:
      timeInterval: 5s
  - name: Jaeger
    type: jaeger
    uid: jaeger
    access: proxy
    url: http://jaeger:16686
"""

DASHBOARDS_YML = """# Generated by agentic_traffic_testing_amd.observability.dashboard
apiVersion: 1
providers:
  - name: agentic-traffic
    orgId: 1
    folder: ""
    type: file
    disableDeletion: false
    updateIntervalSeconds: 30
    allowUiUpdates: true
    options:
      path: /etc/grafana/provisioning/dashboards
"""


def write_all(root: Path, mode: str = "single") -> list[Path]:
    mon = root / "infra" / "monitoring"
    files = {
        mon / "prometheus.yml": prometheus_config("single"),
        mon / "prometheus.distributed.yml": prometheus_config("distributed"),
        mon / "grafana" / "provisioning" / "datasources" / "datasources.yml": DATASOURCES_YML,
        mon / "grafana" / "provisioning" / "dashboards" / "dashboards.yml": DASHBOARDS_YML,
        mon / "grafana" / "provisioning" / "dashboards" / "agentic-traffic.json":
            json.dumps(build_dashboard(), indent=2, ensure_ascii=False) + "\n",
    }
    for p, text in files.items():
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(text)
    return list(files)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Generate the Grafana dashboard + Prometheus config")
    ap.add_argument("--root", default=str(Path(__file__).resolve().parents[2]))
    a = ap.parse_args(argv)
    for p in write_all(Path(a.root)):
        print(f"wrote {p}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
