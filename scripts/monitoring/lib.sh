#!/usr/bin/env bash
# Shared helpers for the monitoring / traffic scripts.

ATTA_ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
INTER_AGENT_SUBNET="${INTER_AGENT_SUBNET:-172.23.0.0/24}"

# Bridge interface (br-<id12>) of the docker network whose name matches $1
# (default: inter_agent).  Prints nothing when it cannot be found.
atta_find_bridge() {
  local pattern="${1:-inter_agent}" nid br
  command -v docker >/dev/null 2>&1 || return 0
  nid="$(docker network ls --filter "name=${pattern}" --format '{{.ID}}' 2>/dev/null | head -n1)"
  [[ -z "${nid}" ]] && return 0
  br="br-${nid:0:12}"
  if ip link show "${br}" >/dev/null 2>&1; then
    echo "${br}"
  fi
}

atta_python() {
  if command -v python3 >/dev/null 2>&1; then echo python3; else echo python; fi
}
