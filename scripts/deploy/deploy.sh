#!/usr/bin/env bash
# Bring up the testbed.  Modes (DEPLOYMENT_MODE in infra/.env or --mode):
#   single       one bridge network (infra/docker-compose.yml)
#   distributed  5 bridges + static IPs (infra/docker-compose.distributed.yml), then the
#                monitoring overlay, host cAdvisor + tcpdump collector, health check, netem
#   multi-vm     per-node `docker compose up` over ssh (NODE1/2/3_HOST), cross-node URLs
# Options: --mode M, --no-monitoring, --no-build, --skip-health
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
load_env
MONITORING="${ENABLE_MONITORING:-1}"; BUILD="--build"; HEALTH=1
while [[ $# -gt 0 ]]; do
  case "$1" in
    --mode) DEPLOYMENT_MODE="$2"; shift 2 ;;
    --no-monitoring) MONITORING=0; shift ;;
    --no-build) BUILD=""; shift ;;
    --skip-health) HEALTH=0; shift ;;
    -h|--help) sed -n '2,8p' "$0"; exit 0 ;;
    *) echo "[!] unknown option $1"; exit 1 ;;
  esac
done
require_docker
CF="$(compose_file)"
echo "============================================================"
echo "Agentic Traffic Testbed (MI355X) - deploy: ${DEPLOYMENT_MODE}"
echo "Compose: ${CF}"
echo "============================================================"

start_monitoring() {
  [[ "${MONITORING}" == "1" ]] || return 0
  echo "[*] Monitoring overlay (Prometheus :9090, Grafana :3001, cAdvisor :8080, mapping :9101)"
  docker compose -f "$(monitoring_file)" up -d ${BUILD}
}

start_collector() {
  # tcp_* collector on the host, exactly once (the reference started it twice)
  if command -v tcpdump >/dev/null 2>&1; then
    mkdir -p "${ROOT_DIR}/logs"
    nohup "${ROOT_DIR}/scripts/monitoring/run_tcpdump.sh" > "${ROOT_DIR}/logs/tcp_collector.log" 2>&1 &
    echo "[*] TCP collector started (pid $!, log logs/tcp_collector.log)"
  else
    echo "[!] tcpdump not installed; tcp_* metrics disabled"
  fi
}

post_up() {
  local llm_health="$1"
  wait_http "${llm_health}" 600 5 || true
  if [[ "${HEALTH}" == "1" ]]; then
    py "${ROOT_DIR}/scripts/monitoring/health_check.py" --compose-file "${CF}" || true
  fi
  if [[ "${ENABLE_NETWORK_EMULATION:-0}" == "1" ]]; then
    "${ROOT_DIR}/scripts/traffic/apply_network_emulation.sh" apply || true
  fi
  "${ROOT_DIR}/scripts/fetch_endpoints.sh" --mode "${DEPLOYMENT_MODE}" || true
}

case "${DEPLOYMENT_MODE}" in
  single)
    docker compose -f "${CF}" up -d ${BUILD}
    start_monitoring
    post_up "http://localhost:8000/health"
    ;;
  distributed)
    docker compose -f "${CF}" up -d ${BUILD}
    start_monitoring
    start_collector
    post_up "http://localhost:8000/health"
    ;;
  multi-vm)
    : "${NODE1_HOST:?NODE1_HOST required}" "${NODE2_HOST:?NODE2_HOST required}" "${NODE3_HOST:?NODE3_HOST required}"
    REMOTE="${REMOTE_REPO_DIR:-/opt/agentic-traffic-testing}"
    SSHU="${SSH_USER:-$USER}"
    LLM_URL="http://${NODE3_HOST}:8000/chat"
    B_URLS="http://${NODE2_HOST}:8102/subtask,http://${NODE2_HOST}:8103/subtask,http://${NODE2_HOST}:8104/subtask,http://${NODE2_HOST}:8105/subtask,http://${NODE2_HOST}:8106/subtask"
    OTEL="http://${NODE1_HOST}:4318/v1/traces"
    remote_up() {  # host, services...
      local host="$1"; shift
      echo "[*] ${host}: docker compose up $*"
      ssh "${SSHU}@${host}" "cd ${REMOTE}/infra && LLM_SERVER_URL=${LLM_URL} AGENT_B_URLS=${B_URLS} OTEL_EXPORTER_OTLP_ENDPOINT=${OTEL} docker compose -f docker-compose.yml up -d ${BUILD} --no-deps $*"
    }
    remote_up "${NODE3_HOST}" llm-backend
    wait_http "http://${NODE3_HOST}:8000/health" 900 10 || true
    remote_up "${NODE2_HOST}" agent-b agent-b-2 agent-b-3 agent-b-4 agent-b-5 mcp-tool-db
    remote_up "${NODE1_HOST}" jaeger agent-a chat-ui
    ;;
esac
echo "[ok] deploy finished (${DEPLOYMENT_MODE})"
