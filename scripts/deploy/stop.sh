#!/usr/bin/env bash
# Stop the testbed.
#   ./scripts/deploy/stop.sh [--mode M] [--volumes] [--networks] [--all]
#   --volumes  also remove named volumes (model cache, Prometheus/Grafana data)
#   --networks remove leftover testbed networks
#   --all      every mode's stack + monitoring + volumes + networks
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
load_env
VOLUMES=""; NETWORKS=0; ALL=0
while [[ $# -gt 0 ]]; do
  case "$1" in
    --mode) DEPLOYMENT_MODE="$2"; shift 2 ;;
    --volumes) VOLUMES="-v"; shift ;;
    --networks) NETWORKS=1; shift ;;
    --all) ALL=1; VOLUMES="-v"; NETWORKS=1; shift ;;
    -h|--help) sed -n '2,7p' "$0"; exit 0 ;;
    *) echo "[!] unknown option $1"; exit 1 ;;
  esac
done
require_docker
down() { [[ -f "$1" ]] && { echo "[*] down: $1"; docker compose -f "$1" down ${VOLUMES} --remove-orphans || true; }; }
if [[ "${ALL}" == "1" ]]; then
  for m in single distributed; do down "$(monitoring_file "${m}")"; done
  for m in single distributed; do down "$(compose_file "${m}")"; done
else
  down "$(monitoring_file)"
  down "$(compose_file)"
fi
if [[ -f "${ROOT_DIR}/logs/tcp_collector.log" ]]; then
  for pid in $(pgrep -x tcpdump 2>/dev/null || true); do
    if tr '\0' ' ' < "/proc/${pid}/cmdline" 2>/dev/null | grep -q "172.23.0.0"; then sudo kill "${pid}" || true; fi
  done
fi
if [[ "${NETWORKS}" == "1" ]]; then
  for n in $(docker network ls --format '{{.Name}}' | grep -E '^infra_(agent-net|agent_a_network|agent_b_network|llm_network|inter_agent_network|tools_network)$' || true); do
    docker network rm "${n}" || true
  done
fi
echo "[ok] stopped"
