#!/usr/bin/env bash
# Print the three mapping tables Grafana joins on: bridge interface -> docker network,
# cgroup scope -> container / compose service, inter-agent IP -> container / service.
# Usage: ./scripts/monitoring/print_network_mappings.sh [network-name]
set -euo pipefail
NET="${1:-${INTER_AGENT_NETWORK:-infra_inter_agent_network}}"
command -v docker >/dev/null 2>&1 || { echo "[!] docker is not installed or not on PATH."; exit 1; }

rule() { printf '%s\n%s\n%s\n' "============================================================" "$1" "============================================================"; }
svc_or_name() { if [[ -z "$2" || "$2" == "<no value>" ]]; then echo "$1"; else echo "$2"; fi; }

rule "Docker bridge interfaces -> Docker networks"
docker network ls --format '{{.ID}} {{.Name}}' | while read -r nid name; do
  br="br-${nid:0:12}"
  ip link show "${br}" >/dev/null 2>&1 && printf '  %-18s -> %s\n' "${br}" "${name}"
done
echo
rule "Containers -> systemd cgroup scopes -> compose services"
docker ps --no-trunc --format '{{.ID}} {{.Names}} {{.Label "com.docker.compose.service"}}' |
  while read -r cid cname csvc; do
    printf '  scope=%-86s container=%-20s service=%s\n' "/system.slice/docker-${cid}.scope" \
      "${cname}" "$(svc_or_name "${cname}" "${csvc:-}")"
  done
echo
rule "Inter-agent network IPs -> containers / services"
if ! docker network inspect "${NET}" >/dev/null 2>&1; then
  echo "[!] Docker network '${NET}' not found. Skipping IP mapping."
  exit 0
fi
printf 'Network: %s\n\n' "${NET}"
docker ps --format '{{.ID}} {{.Names}} {{.Label "com.docker.compose.service"}}' |
  while read -r cid cname csvc; do
    ip_addr="$(docker inspect -f "{{with index .NetworkSettings.Networks \"${NET}\"}}{{.IPAddress}}{{end}}" "${cid}" 2>/dev/null || true)"
    [[ -n "${ip_addr}" ]] && printf '  %-15s -> container=%-20s service=%s\n' "${ip_addr}" "${cname}" \
      "$(svc_or_name "${cname}" "${csvc:-}")"
  done
echo
echo "Done."
