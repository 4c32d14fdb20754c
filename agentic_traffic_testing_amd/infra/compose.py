"""Docker Compose topology generator.

The reference hand-maintains four compose files (infra/docker-compose.yml,
docker-compose.distributed.yml, docker-compose.monitoring.yml,
docker-compose.monitoring.distributed.yml) whose services differ only in addressing.  Here
one service table drives all of them, so hostnames, ports, static IPs and env knobs cannot
drift apart:

* single mode - one bridge ``agent-net``, compose DNS names;
* distributed mode - five bridges (agent_a 172.20, agent_b 172.21, llm 172.22,
  inter_agent 172.23, tools 172.24), every service on its home network plus
  ``inter_agent_network`` with the static IPs the TCP collector's ``SERVICE_IPS`` expects,
  ``extra_hosts`` pinning peer names to inter-agent IPs;
* monitoring overlays (Prometheus 9090, Grafana 3001, cAdvisor 8080, mapping exporter 9101;
  distributed variant pins 172.23.0.70-.73 and joins the external inter-agent network).

MI355X specifics: the LLM service is the ROCm image (``llm/Dockerfile``) with
``/dev/kfd`` + ``/dev/dri`` device mappings, ``video``/``render`` groups, host IPC (TP
ranks share the RCCL / shm step channel) and ``HIP_VISIBLE_DEVICES`` instead of the
reference's NVIDIA runtime reservation; ``LLM_TENSOR_PARALLEL_SIZE`` selects TP.
Fixes: the LLM health check start period is 600 s in both modes (the reference uses 10 s
in distributed mode, which marks a loading backend unhealthy), and the agents' docker
image no longer installs the LLM stack.

``python -m agentic_traffic_testing_amd.infra.compose`` rewrites the files under infra/.
"""
from __future__ import annotations

import argparse
from pathlib import Path

import yaml

N_AGENT_B = 5
AGENT_B_PORT0 = 8102

NETWORKS = {  # name: (subnet env, default subnet)
    "agent_a_network": ("NETWORK_AGENT_A_SUBNET", "172.20.0.0/24"),
    "agent_b_network": ("NETWORK_AGENT_B_SUBNET", "172.21.0.0/24"),
    "llm_network": ("NETWORK_LLM_SUBNET", "172.22.0.0/24"),
    "inter_agent_network": ("NETWORK_INTER_AGENT_SUBNET", "172.23.0.0/24"),
    "tools_network": ("NETWORK_TOOLS_SUBNET", "172.24.0.0/24"),
}


def _b_name(i: int) -> str:
    return "agent-b" if i == 1 else f"agent-b-{i}"


def _b_env_prefix(i: int) -> str:
    return "AGENT_B" if i == 1 else f"AGENT_B_{i}"


def inter_ips() -> dict:
    """service -> (env var, default inter-agent IP)."""
    ips = {"agent-a": ("AGENT_A_INTER_IP", "172.23.0.10"),
           "llm-backend": ("LLM_BACKEND_INTER_IP", "172.23.0.30"),
           "mcp-tool-db": ("MCP_TOOL_DB_INTER_IP", "172.23.0.40"),
           "chat-ui": ("CHAT_UI_IP", "172.23.0.50"),
           "jaeger": ("JAEGER_IP", "172.23.0.60")}
    for i in range(1, N_AGENT_B + 1):
        ips[_b_name(i)] = (f"{_b_env_prefix(i)}_INTER_IP", f"172.23.0.{19 + i}")
    return ips


HOME = {  # service -> (home network, env var, default home IP)
    "agent-a": ("agent_a_network", "AGENT_A_IP", "172.20.0.10"),
    "llm-backend": ("llm_network", "LLM_BACKEND_IP", "172.22.0.10"),
    "mcp-tool-db": ("tools_network", "MCP_TOOL_DB_IP", "172.24.0.10"),
}
for _i in range(1, N_AGENT_B + 1):
    HOME[_b_name(_i)] = ("agent_b_network", f"{_b_env_prefix(_i)}_IP", f"172.21.0.{9 + _i}")


def _ip(svc: str) -> str:
    env, default = inter_ips()[svc]
    return f"${{{env}:-{default}}}"


def _common_llm_env() -> list:
    keys = [("LOG_LLM_REQUESTS", "0"), ("LLM_LOG_MAX_CHARS", "500"), ("LLM_DTYPE", "bfloat16"),
            ("LLM_MAX_NUM_SEQS", "12"), ("LLM_MAX_NUM_BATCHED_TOKENS", "8192"),
            ("LLM_MAX_TOKENS", "512"), ("LLM_GPU_MEMORY_UTILIZATION", "0.90"),
            ("LLM_MAX_MODEL_LEN", "4096"), ("LLM_PROMPT_SAFETY_MARGIN_TOKENS", "128"),
            ("LLM_METRICS_ENABLED", "1"), ("LLM_METRICS_INCLUDE_TOKENS", "1"),
            ("LLM_METRICS_PREFIX", "llm"), ("LLM_TENSOR_PARALLEL_SIZE", "1"),
            ("LLM_LOAD_FORMAT", "auto"), ("LLM_DATA_PARALLEL_SIZE", "1"),
            ("LLM_QUANTIZATION", ""),
            ("LLM_MODEL", "meta-llama/Llama-3.1-8B-Instruct")]
    return [f"{k}=${{{k}:-{v}}}" for k, v in keys]


def llm_service(distributed: bool) -> dict:
    env = ["NODE_NAME=node3_llm", "HF_TOKEN=${HF_TOKEN:-}",
           "HUGGINGFACE_HUB_TOKEN=${HUGGINGFACE_HUB_TOKEN:-${HF_TOKEN:-}}",
           "HIP_VISIBLE_DEVICES=${HIP_VISIBLE_DEVICES:-0}",
           "HSA_ENABLE_IPC_MODE_LEGACY=0",
           "OTEL_EXPORTER_OTLP_ENDPOINT="
           + (f"http://{_ip('jaeger')}:4318/v1/traces" if distributed
              else "${OTEL_EXPORTER_OTLP_ENDPOINT:-http://jaeger:4318/v1/traces}"),
           ] + _common_llm_env()
    svc = {
        "build": {"context": "..", "dockerfile": "llm/Dockerfile"},
        "container_name": "llm-backend",
        "environment": env,
        "command": ["python3", "-m", "llm.serve_llm", "--host", "0.0.0.0", "--port", "8000",
                    "--model", "${LLM_MODEL:-meta-llama/Llama-3.1-8B-Instruct}",
                    "--max-model-len", "${LLM_MAX_MODEL_LEN:-4096}",
                    "--dtype", "${LLM_DTYPE:-bfloat16}",
                    "--max-num-seqs", "${LLM_MAX_NUM_SEQS:-12}",
                    "--max-num-batched-tokens", "${LLM_MAX_NUM_BATCHED_TOKENS:-8192}",
                    "--gpu-memory-utilization", "${LLM_GPU_MEMORY_UTILIZATION:-0.90}",
                    "--tensor-parallel-size", "${LLM_TENSOR_PARALLEL_SIZE:-1}",
                    "--data-parallel-size", "${LLM_DATA_PARALLEL_SIZE:-1}"],
        "volumes": ["hf_model_cache:/root/.cache/huggingface"],
        "ports": ["8000:8000"],
        # ROCm device access (replaces the NVIDIA runtime reservation)
        "devices": ["/dev/kfd", "/dev/dri"],
        "group_add": ["video", "render"],
        "security_opt": ["seccomp=unconfined"],
        "ipc": "host",
        "shm_size": "16g",
        "healthcheck": {
            "test": ["CMD", "python3", "-c", "import urllib.request; urllib.request.urlopen("
                     "'http://localhost:8000/health', timeout=2).read()"],
            "interval": "15s", "timeout": "3s", "retries": 40, "start_period": "600s"},
    }
    if distributed:
        svc["hostname"] = "llm-backend"
    return svc


def agent_a_service(distributed: bool) -> dict:
    if distributed:
        llm_url = f"http://{_ip('llm-backend')}:8000/chat"
        b_urls = ",".join(f"http://{_ip(_b_name(i))}:{AGENT_B_PORT0 + i - 1}/subtask"
                          for i in range(1, N_AGENT_B + 1))
        otel = f"http://{_ip('jaeger')}:4318/v1/traces"
    else:
        llm_url = "${LLM_SERVER_URL:-http://llm-backend:8000/chat}"
        b_urls = "${AGENT_B_URLS:-" + ",".join(
            f"http://{_b_name(i)}:{AGENT_B_PORT0 + i - 1}/subtask"
            for i in range(1, N_AGENT_B + 1)) + "}"
        otel = "${OTEL_EXPORTER_OTLP_ENDPOINT:-http://jaeger:4318/v1/traces}"
    return {
        "build": {"context": "..", "dockerfile": "agents/Dockerfile"},
        "container_name": "agent-a",
        "environment": [f"LLM_SERVER_URL={llm_url}", "NODE_NAME=node1_agentA",
                        "AGENT_A_PORT=8101", "OTEL_SERVICE_NAME=agent-a",
                        f"OTEL_EXPORTER_OTLP_ENDPOINT={otel}", f"AGENT_B_URLS={b_urls}",
                        "LLM_TIMEOUT_SECONDS=${LLM_TIMEOUT_SECONDS:-120}",
                        "AGENT_B_TIMEOUT_SECONDS=${AGENT_B_TIMEOUT_SECONDS:-120}",
                        "LOG_LLM_REQUESTS=${LOG_LLM_REQUESTS:-0}",
                        "LLM_LOG_MAX_CHARS=${LLM_LOG_MAX_CHARS:-500}"],
        "depends_on": {"llm-backend": {"condition": "service_healthy"}},
        "ports": ["8101:8101"],
        "command": ["python", "-m", "agents.agent_a.server"],
        "volumes": ["../logs:/app/logs"],
        "cap_add": ["NET_ADMIN"],
    }


def agent_b_service(i: int, distributed: bool) -> dict:
    port = AGENT_B_PORT0 + i - 1
    llm_url = (f"http://{_ip('llm-backend')}:8000/chat" if distributed
               else "${LLM_SERVER_URL:-http://llm-backend:8000/chat}")
    otel = (f"http://{_ip('jaeger')}:4318/v1/traces" if distributed
            else "${OTEL_EXPORTER_OTLP_ENDPOINT:-http://jaeger:4318/v1/traces}")
    node = "node2_agentB" if i == 1 else f"node2_agentB_{i}"
    return {
        "build": {"context": "..", "dockerfile": "agents/Dockerfile"},
        "container_name": _b_name(i),
        "environment": [f"LLM_SERVER_URL={llm_url}", f"NODE_NAME={node}",
                        f"AGENT_B_PORT={port}", f"OTEL_SERVICE_NAME=agent-b-{i}",
                        f"OTEL_EXPORTER_OTLP_ENDPOINT={otel}",
                        "LLM_TIMEOUT_SECONDS=${LLM_TIMEOUT_SECONDS:-120}",
                        "LOG_LLM_REQUESTS=${LOG_LLM_REQUESTS:-0}",
                        "LLM_LOG_MAX_CHARS=${LLM_LOG_MAX_CHARS:-500}"],
        "depends_on": {"llm-backend": {"condition": "service_healthy"}},
        "ports": [f"{port}:{port}"],
        "command": ["python", "-m", "agents.agent_b.server"],
        "volumes": ["../logs:/app/logs"],
        "cap_add": ["NET_ADMIN"],
    }


def tool_db_service() -> dict:
    return {"build": {"context": "..", "dockerfile": "tools/mcp_tool_db/Dockerfile"},
            "container_name": "mcp-tool-db",
            "environment": ["NODE_NAME=node4_toolDB", "MCP_TOOL_DB_PORT=8201"],
            "ports": ["8201:8201"]}


def ui_service() -> dict:
    return {"build": {"context": "..", "dockerfile": "ui/Dockerfile"},
            "container_name": "chat-ui", "ports": ["3000:3000"],
            "depends_on": ["agent-a", "agent-b"]}


def jaeger_service() -> dict:
    return {"image": "jaegertracing/all-in-one:1.57", "container_name": "jaeger",
            "ports": ["16686:16686", "4317:4317", "4318:4318"]}


def services(distributed: bool) -> dict:
    s = {"llm-backend": llm_service(distributed), "agent-a": agent_a_service(distributed)}
    for i in range(1, N_AGENT_B + 1):
        s[_b_name(i)] = agent_b_service(i, distributed)
    s["mcp-tool-db"] = tool_db_service()
    s["chat-ui"] = ui_service()
    s["jaeger"] = jaeger_service()
    return s


def single_compose() -> dict:
    s = services(False)
    for v in s.values():
        v["networks"] = ["agent-net"]
    return {"services": s, "networks": {"agent-net": {"driver": "bridge"}},
            "volumes": {"hf_model_cache": {}}}


def distributed_compose() -> dict:
    s = services(True)
    ips = inter_ips()
    peers = ["llm-backend"] + [_b_name(i) for i in range(1, N_AGENT_B + 1)] + ["jaeger"]
    for name, v in s.items():
        v["hostname"] = name
        nets = {}
        if name in HOME:
            net, env, default = HOME[name]
            nets[net] = {"ipv4_address": f"${{{env}:-{default}}}"}
        env, default = ips[name]
        nets["inter_agent_network"] = {"ipv4_address": f"${{{env}:-{default}}}"}
        v["networks"] = nets
        if name.startswith("agent-"):
            v["extra_hosts"] = [f"{p}:{_ip(p)}" for p in peers if p != name]
        if name == "chat-ui":
            v["extra_hosts"] = [f"agent-a:{_ip('agent-a')}"]
    nets = {n: {"driver": "bridge", "ipam": {"config": [{"subnet": f"${{{e}:-{d}}}"}]}}
            for n, (e, d) in NETWORKS.items()}
    return {"services": s, "networks": nets, "volumes": {"hf_model_cache": {}}}


def monitoring_compose(distributed: bool) -> dict:
    prom_cfg = "prometheus.distributed.yml" if distributed else "prometheus.yml"
    s = {
        "prometheus": {
            "image": "prom/prometheus:v2.47.0", "container_name": "prometheus",
            "hostname": "prometheus",
            "volumes": [f"./monitoring/{prom_cfg}:/etc/prometheus/prometheus.yml:ro",
                        "prometheus_data:/prometheus"],
            "command": ["--config.file=/etc/prometheus/prometheus.yml",
                        "--storage.tsdb.path=/prometheus", "--web.enable-lifecycle",
                        "--storage.tsdb.retention.time=7d"],
            "ports": ["9090:9090"], "restart": "unless-stopped",
            "extra_hosts": ["host.docker.internal:host-gateway"]},
        "grafana": {
            "image": "grafana/grafana:10.2.0", "container_name": "grafana",
            "hostname": "grafana",
            "environment": ["GF_SECURITY_ADMIN_USER=admin", "GF_SECURITY_ADMIN_PASSWORD=admin",
                            "GF_USERS_ALLOW_SIGN_UP=false", "GF_SERVER_HTTP_PORT=3001",
                            "GF_AUTH_ANONYMOUS_ENABLED=true",
                            "GF_AUTH_ANONYMOUS_ORG_ROLE=Viewer"],
            "volumes": ["./monitoring/grafana/provisioning:/etc/grafana/provisioning:ro",
                        "grafana_data:/var/lib/grafana"],
            "ports": ["3001:3001"], "depends_on": ["prometheus"], "restart": "unless-stopped"},
        "cadvisor": {
            "image": "gcr.io/cadvisor/cadvisor:v0.47.2", "container_name": "cadvisor",
            "hostname": "cadvisor", "privileged": True,
            "command": ["--docker_only=true", "--store_container_labels=true"],
            "volumes": ["/:/rootfs:ro", "/var/run:/var/run:ro", "/sys:/sys:ro",
                        "/var/lib/docker/:/var/lib/docker:ro", "/dev/disk/:/dev/disk:ro"],
            "ports": ["8080:8080"], "restart": "unless-stopped"},
        "docker-mapping-exporter": {
            "build": {"context": "..", "dockerfile": "scripts/monitoring/Dockerfile.exporter"},
            "container_name": "docker-mapping-exporter", "hostname": "docker-mapping-exporter",
            "environment": ["EXPORTER_PORT=9101",
                            "INTER_AGENT_NETWORK=${INTER_AGENT_NETWORK:-infra_inter_agent_network}"],
            "volumes": ["/var/run/docker.sock:/var/run/docker.sock:ro"],
            "ports": ["9101:9101"], "restart": "unless-stopped"},
        "ebpf-exporter": {
            "image": "ghcr.io/cloudflare/ebpf_exporter:v2.4.2", "container_name": "ebpf-exporter",
            "privileged": True, "pid": "host", "profiles": ["ebpf"],
            "command": ["--config.dir=/config", "--config.names=tcp"],
            "volumes": ["./monitoring/ebpf_exporter:/config:ro",
                        "/sys/kernel/debug:/sys/kernel/debug:ro"],
            "ports": ["9435:9435"], "restart": "unless-stopped"},
    }
    if distributed:
        for i, name in enumerate(("prometheus", "grafana", "cadvisor",
                                  "docker-mapping-exporter", "ebpf-exporter")):
            s[name]["networks"] = {"inter_agent_network": {"ipv4_address": f"172.23.0.{70 + i}"}}
        nets = {"inter_agent_network": {"external": True, "name": "infra_inter_agent_network"}}
    else:
        for v in s.values():
            v["networks"] = ["agent-net"]
        nets = {"agent-net": {"external": True, "name": "infra_agent-net"}}
    return {"services": s, "networks": nets,
            "volumes": {"prometheus_data": {}, "grafana_data": {}}}


HEADER = ("# Generated by agentic_traffic_testing_amd/infra/compose.py - edit the generator,\n"
          "# then: python -m agentic_traffic_testing_amd.infra.compose\n")


def write_all(root: Path) -> list[Path]:
    infra = root / "infra"
    infra.mkdir(parents=True, exist_ok=True)
    files = {infra / "docker-compose.yml": single_compose(),
             infra / "docker-compose.distributed.yml": distributed_compose(),
             infra / "docker-compose.monitoring.yml": monitoring_compose(False),
             infra / "docker-compose.monitoring.distributed.yml": monitoring_compose(True)}
    for p, doc in files.items():
        p.write_text(HEADER + yaml.safe_dump(doc, sort_keys=False, width=120))
    return list(files)


def main(argv: list[str] | None = None) -> int:
    ap = argparse.ArgumentParser(description="Generate the docker compose topologies")
    ap.add_argument("--root", default=str(Path(__file__).resolve().parents[2]))
    a = ap.parse_args(argv)
    for p in write_all(Path(a.root)):
        print(f"wrote {p}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
