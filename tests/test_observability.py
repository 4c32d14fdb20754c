"""Observability + infra plane (§5.5 metric contracts)."""
import json
import struct
import threading
from http.server import HTTPServer
from pathlib import Path

import httpx
import pytest
import yaml

from agentic_traffic_testing_amd.infra import compose, endpoints
from agentic_traffic_testing_amd.observability import dashboard, docker_mapping_exporter as dme
from agentic_traffic_testing_amd.observability import health_check, tcp_collector as tc
from agentic_traffic_testing_amd.observability import traffic_analysis as ta

ROOT = Path(__file__).resolve().parents[1]


def _line(ts, src, sport, dst, dport, flags, length=0):
    return f"{ts:.6f} IP {src}.{sport} > {dst}.{dport}: Flags [{flags}], seq 1, length {length}"


A, LLM = "172.23.0.10", "172.23.0.30"


def _handshake_flow(agg, t0=1000.0, port=40000, payload=900):
    lines = [_line(t0, A, port, LLM, 8000, "S"),
             _line(t0 + 0.0004, LLM, 8000, A, port, "S."),
             _line(t0 + 0.0005, A, port, LLM, 8000, "."),
             _line(t0 + 0.01, A, port, LLM, 8000, "P.", payload),
             _line(t0 + 0.30, LLM, 8000, A, port, "P.", 2000),
             _line(t0 + 0.31, LLM, 8000, A, port, "F."),
             _line(t0 + 0.32, A, port, LLM, 8000, "F.")]
    for ln in lines:
        assert agg.ingest(ln)
    assert not agg.ingest("garbage line")


def _series(text, name):
    return {ln.split(" ")[0]: float(ln.split(" ")[1]) for ln in text.splitlines()
            if ln.startswith(name + "{") or ln.startswith(name + " ")}


def test_tcp_collector_contract():
    agg = tc.TcpAggregator()
    _handshake_flow(agg)
    txt = agg.render()
    pk = _series(txt, "tcp_packets_total")
    assert pk['tcp_packets_total{src_service="agent_a",dst_service="llm_backend"}'] == 4
    assert pk['tcp_packets_total{src_service="llm_backend",dst_service="agent_a"}'] == 3
    by = _series(txt, "tcp_bytes_total")
    assert by['tcp_bytes_total{src_service="agent_a",dst_service="llm_backend"}'] == 900
    assert _series(txt, "tcp_syn_total") == {
        'tcp_syn_total{src_service="agent_a",dst_service="llm_backend"}': 1}
    rtt = _series(txt, "tcp_rtt_handshake_seconds_bucket")
    key = 'tcp_rtt_handshake_seconds_bucket{src_service="agent_a",dst_service="llm_backend",le='
    assert rtt[key + '"0.0005"}'] == 1 and rtt[key + '"inf"}'] == 1
    dur = _series(txt, "tcp_flow_duration_seconds_bucket")
    dkey = 'tcp_flow_duration_seconds_bucket{src_service="agent_a",dst_service="llm_backend",le='
    assert dur[dkey + '"0.1"}'] == 0 and dur[dkey + '"0.5"}'] == 1  # once, at the first FIN
    assert dur[dkey + '"inf"}'] == 1
    sizes = _series(txt, "tcp_packet_size_bytes_bucket")
    assert sizes['tcp_packet_size_bytes_bucket{le="64"}'] == 5
    assert sizes['tcp_packet_size_bytes_bucket{le="inf"}'] == 7
    assert "# TYPE tcp_flow_duration_seconds_bucket counter" in txt
    assert "_sum" not in txt and "_count" not in txt
    assert _series(txt, "tcp_flows_active")["tcp_flows_active"] == 1
    # idle eviction on packet time: does not observe the duration a second time
    assert agg.sweep(max_idle=60.0, now=1000.0 + 120) == 1
    dur = _series(agg.render(), "tcp_flow_duration_seconds_bucket")
    assert dur[dkey + '"inf"}'] == 1


def test_tcp_collector_legacy_double_count_and_external():
    agg = tc.TcpAggregator(legacy=True)
    _handshake_flow(agg)
    agg.sweep(max_idle=60.0, now=2000.0)
    dur = _series(agg.render(), "tcp_flow_duration_seconds_bucket")
    dkey = 'tcp_flow_duration_seconds_bucket{src_service="agent_a",dst_service="llm_backend",le='
    assert dur[dkey + '"inf"}'] == 3  # 2 FINs + eviction, as the reference counts
    agg2 = tc.TcpAggregator()
    agg2.ingest(_line(1.0, "10.0.0.1", 1, "10.0.0.2", 2, "S"))
    assert 'src_service="external",dst_service="external"' in agg2.render()


def test_tcp_collector_http():
    agg = tc.TcpAggregator()
    _handshake_flow(agg)
    srv = HTTPServer(("127.0.0.1", 0), tc.make_handler(agg))
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    try:
        base = f"http://127.0.0.1:{srv.server_address[1]}"
        assert "tcp_bytes_total" in httpx.get(base + "/metrics").text
        assert httpx.get(base + "/health").text == "OK"
        assert httpx.get(base + "/x").status_code == 404
    finally:
        srv.shutdown()
        srv.server_close()


class FakeDocker:
    def get(self, path):
        if path == "/networks":
            return [{"Id": "abcdef1234567890", "Name": "infra_inter_agent_network",
                     "Driver": "bridge"}, {"Id": "ff", "Name": "host", "Driver": "host"}]
        if path == "/containers/json":
            return [{"Id": "c" * 64, "Names": ["/agent-a"],
                     "Labels": {"com.docker.compose.service": "agent-a"},
                     "NetworkSettings": {"Networks": {"infra_inter_agent_network":
                                                      {"IPAddress": "172.23.0.10"}}}},
                    {"Id": "d" * 64, "Names": ["/weird\"name"], "Labels": {}}]
        return None


def test_docker_mapping_exporter():
    txt = dme.MappingExporter(api=FakeDocker(), inter_agent_network="infra_inter_agent_network",
                              ttl=0).render()
    assert ('docker_network_mapping{interface="br-abcdef123456",'
            'network_name="infra_inter_agent_network"} 1') in txt
    assert (f'docker_container_mapping{{id="/system.slice/docker-{"c" * 64}.scope",'
            'container_name="agent-a",service_name="agent-a"} 1') in txt
    assert ('docker_ip_mapping{ip_address="172.23.0.10",container_name="agent-a",'
            'service_name="agent-a"} 1') in txt
    assert 'container_name="weird\\"name"' in txt


def _pcap(tmp_path, linktype=1):
    def tcp_frame(src, dst, sport, dport, flags, payload=b""):
        tcp = struct.pack("!HHIIBBHHH", sport, dport, 1, 0, 5 << 4, flags, 1000, 0, 0) + payload
        ip = struct.pack("!BBHHHBBH4s4s", 0x45, 0, 20 + len(tcp), 0, 0, 64, 6, 0,
                         bytes(map(int, src.split("."))), bytes(map(int, dst.split("."))))
        if linktype == 1:
            return b"\x00" * 12 + b"\x08\x00" + ip + tcp
        return b"\x00" * 14 + b"\x08\x00" + ip + tcp  # Linux cooked v1
    frames = [(0.0, tcp_frame(A, LLM, 5000, 8000, 0x02)),
              (0.001, tcp_frame(LLM, A, 8000, 5000, 0x12)),
              (0.5, tcp_frame(A, LLM, 5000, 8000, 0x18, b"x" * 100)),
              (1.5, tcp_frame(LLM, A, 8000, 5000, 0x11)),
              (1.6, tcp_frame("172.23.0.20", LLM, 6000, 8000, 0x04))]
    out = struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65535, linktype)
    for ts, fr in frames:
        out += struct.pack("<IIII", 1700000000 + int(ts), int((ts % 1) * 1e6), len(fr), len(fr)) + fr
    p = tmp_path / f"cap{linktype}.pcap"
    p.write_bytes(out)
    return p


@pytest.mark.parametrize("linktype", [1, 113])
def test_traffic_analysis_pcap(tmp_path, linktype):
    res = ta.analyze_pcap(_pcap(tmp_path, linktype))
    assert res["total_packets"] == 5 and res["total_flows"] == 2
    assert res["duration_seconds"] == pytest.approx(1.6, abs=1e-5)
    pair = res["service_pairs"][("agent-a", "llm-backend")][0]
    assert pair.syn_count == 2 and pair.fin_count == 1 and pair.packet_count == 4
    assert res["connections_per_second"] == {0: 2}
    assert res["service_pairs"][("agent-b-1", "llm-backend")][0].rst_count == 1
    files = ta.export_csv(res, tmp_path / "out")
    assert [f.name for f in files] == ["flows.csv", "timeseries.csv"]
    assert "TRAFFIC FLOW SUMMARY" in ta.flow_summary(res)


def test_traffic_analysis_telemetry(tmp_path):
    (tmp_path / "n_AgentA.log").write_text(
        json.dumps({"task_id": "t1", "event_type": "task_received", "timestamp_ms": 2}) + "\n"
        + json.dumps({"task_id": "t1", "event_type": "llm_request", "timestamp_ms": 1}) + "\nbad\n")
    t = ta.analyze_telemetry(tmp_path)
    assert t["total_events"] == 2 and [e["event_type"] for e in t["tasks"]["t1"]] == [
        "llm_request", "task_received"]


CONTRACT_TITLES = [
    "Active Containers (Docker)", "Docker Network TX Rate", "Docker Network RX Rate",
    "LLM Request Rate — success vs error", "Network Transmit Rate by Interface",
    "Network Receive Rate by Interface", "Packets Transmitted (by Interface)",
    "Packets per Minute (by Interface)", "CPU (core equivalents per container)",
    "Memory Usage per container", "TCP Bytes/s by Service Pair", "TCP Bytes/s from LLM Backend",
    "TCP RTT (SYN/SYN-ACK Agent A → LLM)", "TCP Flow Duration (Agent A → LLM)",
    "LLM End-to-end Latency (p50/p95)", "LLM Time-to-First-Token (TTFT p50/p95)",
    "Prompt Tokens / s", "Completion Tokens / s", "In-flight LLM Requests",
    "LLM Tokens & In-flight Requests (overlay)", "KV-cache-limited max concurrency",
    "vLLM max_num_batched_tokens", "Max tokens per generation (LLM_MAX_TOKENS)",
    "GPU memory utilization target", "LLM Errors — total (since restart)",
    "LLM Errors — last 1 h", "Free Concurrent Slots (KV-cache capacity − in-flight)",
    "LLM Interarrival Time (30s rolling avg)", "Request arrivals in last 4s (by status)",
    "LLM Request Rate — success vs error (30s window)",
    "Concurrent In-flight Requests (burst signature)", "Interarrival Jitter (p95 − p50)",
    "Queue Wait Distribution (p50/p95/p99) + In-flight",
    "Burstiness Coefficient (peak 10s / avg 5m)"]


def test_dashboard_contract():
    d = dashboard.build_dashboard()
    assert d["uid"] == "agentic-traffic-testbed" and d["refresh"] == "5s"
    titles = [p["title"] for p in d["panels"] if p["type"] != "row"]
    for t in CONTRACT_TITLES:
        assert t in titles, t
    rows = [p["title"] for p in d["panels"] if p["type"] == "row"]
    assert rows[:8] == ["Overview", "Network Traffic", "Resource Usage",
                        "Service-level Network (TCP)", "AI Performance (LLM)",
                        "LLM Configuration", "Interarrival Interpretation",
                        "Traffic Characterization"]
    ids = [p["id"] for p in d["panels"]]
    assert len(ids) == len(set(ids))
    ys = [p["gridPos"]["y"] for p in d["panels"]]
    assert ys == sorted(ys)  # rows and panels in reading order
    exprs = [t["expr"] for p in d["panels"] for t in p.get("targets", [])]
    assert ("max_over_time(rate(llm_requests_total[10s])[5m:10s]) / "
            "rate(llm_requests_total[5m])") in exprs
    # the committed JSON is the generator's output
    committed = json.loads((ROOT / "infra/monitoring/grafana/provisioning/dashboards/"
                                   "agentic-traffic.json").read_text())
    assert committed == json.loads(json.dumps(d, ensure_ascii=False))


def test_prometheus_config():
    cfg = yaml.safe_load(dashboard.prometheus_config())
    jobs = {j["job_name"]: j for j in cfg["scrape_configs"]}
    assert set(jobs) == {"prometheus", "cadvisor", "tcp-metrics", "llm-backend", "docker-mapping"}
    assert jobs["llm-backend"]["scrape_interval"] == "2s"
    assert cfg["global"]["scrape_interval"] == "5s"


def test_compose_topologies():
    single = compose.single_compose()
    dist = compose.distributed_compose()
    names = {"llm-backend", "agent-a", "agent-b", "agent-b-2", "agent-b-3", "agent-b-4",
             "agent-b-5", "mcp-tool-db", "chat-ui", "jaeger"}
    assert set(single["services"]) == names == set(dist["services"])
    llm = single["services"]["llm-backend"]
    assert "/dev/kfd" in llm["devices"] and "deploy" not in llm
    ports = sorted(int(p.split(":")[0]) for s in single["services"].values()
                   for p in s.get("ports", []))
    assert ports == [3000, 4317, 4318, 8000, 8101, 8102, 8103, 8104, 8105, 8106, 8201, 16686]
    # distributed static IPs are exactly the collector's SERVICE_IPS (inter-agent net)
    got = {}
    for name, svc in dist["services"].items():
        ip = svc["networks"]["inter_agent_network"]["ipv4_address"]
        got[ip.split(":-")[1].rstrip("}")] = name.replace("-", "_")
    for ip, svc in tc.SERVICE_IPS.items():
        if ip.startswith("172.23."):
            name = "agent_b_1" if got[ip] == "agent_b" else got[ip]
            assert name == svc, (ip, name, svc)
    assert set(dist["networks"]) == {"agent_a_network", "agent_b_network", "llm_network",
                                     "inter_agent_network", "tools_network"}
    mon = compose.monitoring_compose(True)
    assert mon["services"]["prometheus"]["networks"]["inter_agent_network"][
        "ipv4_address"] == "172.23.0.70"
    # committed files are the generator's output
    for fname, doc in (("docker-compose.yml", single), ("docker-compose.distributed.yml", dist)):
        assert yaml.safe_load((ROOT / "infra" / fname).read_text()) == json.loads(json.dumps(doc))


def test_endpoints_summary():
    rows = [{"Service": "llm-backend", "State": "running",
             "Publishers": [{"PublishedPort": 8000, "TargetPort": 8000}]},
            {"Service": "agent-b-3", "State": "running",
             "Publishers": [{"PublishedPort": 8104, "TargetPort": 8104},
                            {"PublishedPort": 0, "TargetPort": 9}]}]
    e = endpoints.summarize(rows)
    assert e[0]["urls"] == ["http://localhost:8104/subtask"]
    assert e[1]["urls"][0] == "http://localhost:8000/chat"
    assert "-L 8000:localhost:8000 -L 8104:localhost:8104" in endpoints.render(e)


def test_health_check_against_stack(tmp_path):
    from agentic_traffic_testing_amd.testing.stack import Stack, cpu_engine

    eng = cpu_engine(max_model_len=1024, num_kv_blocks=256, max_num_batched_tokens=1024)
    with Stack(eng, n_agent_b=2, log_dir=str(tmp_path), env={"LLM_MAX_TOKENS": "4"}) as s:
        s.llm.state.s.max_tokens = 4
        b_urls = ",".join(u + "/subtask" for _, u in s.agent_b)
        args = ["--skip-docker", "--skip-monitoring", "--json", "--llm-url", s.llm.url + "/chat",
                "--agent-a-url", s.agent_a_url + "/task", "--agent-b-urls", b_urls,
                "--ui-url", "http://127.0.0.1:9/"]
        rep = health_check.run_checks(health_check.make_parser().parse_args(args))
        assert rep.passed, [c for c in rep.checks if not c.ok]
        names = [c.name for c in rep.checks]
        assert "Agent A can reach LLM" in names and "Agent B (2) can reach LLM" in names
        ui = [c for c in rep.checks if c.name == "UI endpoint"][0]
        assert not ui.ok and not ui.critical
        bad = health_check.run_checks(health_check.make_parser().parse_args(
            ["--skip-docker", "--skip-monitoring", "--json", "--llm-url",
             "http://127.0.0.1:9/chat", "--agent-a-url", "http://127.0.0.1:9/task",
             "--agent-b-urls", "http://127.0.0.1:9/subtask"]))
        assert not bad.passed
