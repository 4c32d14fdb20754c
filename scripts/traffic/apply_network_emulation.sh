#!/usr/bin/env bash
# tc/netem impairment of the agent containers (fault/impairment injection).
#
#   ./scripts/traffic/apply_network_emulation.sh [apply|remove|status] [--containers "a b"]
#
# Reads NETWORK_DELAY_MS (10), NETWORK_JITTER_MS (2), NETWORK_LOSS_PERCENT (0) and
# NETEM_INTERFACE (eth0) from the environment or infra/.env.  ``apply`` uses
# ``tc qdisc replace ... root netem delay Dms Jms [loss L%]`` inside each running
# container (needs cap NET_ADMIN, granted in the compose files) and fails when no
# container could be impaired.  The LLM container is not impaired by default, as in the
# reference; add it with --containers to emulate a remote backend.
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
ENV_FILE="${ROOT}/infra/.env"
if [[ -f "${ENV_FILE}" ]]; then
  set -a
  # shellcheck disable=SC1090
  source <(grep -Ev '^\s*(#|$)' "${ENV_FILE}")
  set +a
fi
DELAY_MS="${NETWORK_DELAY_MS:-10}"
JITTER_MS="${NETWORK_JITTER_MS:-2}"
LOSS_PERCENT="${NETWORK_LOSS_PERCENT:-0}"
IFACE="${NETEM_INTERFACE:-eth0}"
CONTAINERS="${NETEM_CONTAINERS:-agent-a agent-b agent-b-2 agent-b-3 agent-b-4 agent-b-5}"

ACTION="${1:-apply}"
shift || true
while [[ $# -gt 0 ]]; do
  case "$1" in
    --containers) CONTAINERS="$2"; shift 2 ;;
    --interface) IFACE="$2"; shift 2 ;;
    *) echo "unknown option: $1" >&2; exit 2 ;;
  esac
done

running() { docker ps --format '{{.Names}}' | grep -qx "$1"; }

netem_spec() {
  local spec="delay ${DELAY_MS}ms ${JITTER_MS}ms"
  [[ "${LOSS_PERCENT}" != "0" ]] && spec="${spec} loss ${LOSS_PERCENT}%"
  echo "${spec}"
}

case "${ACTION}" in
  apply)
    echo "[*] netem: $(netem_spec) on ${IFACE} of: ${CONTAINERS}"
    tried=0; applied=0
    for c in ${CONTAINERS}; do
      if ! running "${c}"; then echo "    [!] ${c} not running, skipping."; continue; fi
      tried=1
      # shellcheck disable=SC2046
      if docker exec "${c}" tc qdisc replace dev "${IFACE}" root netem $(netem_spec) 2>/dev/null; then
        applied=1; echo "    [ok] ${c}"
      else
        echo "    [!] ${c}: tc failed (missing NET_ADMIN or iproute2?)"
      fi
    done
    if [[ ${tried} -eq 0 ]]; then echo "[!] No running agent containers found."; exit 1; fi
    if [[ ${applied} -eq 0 ]]; then echo "[!] Network emulation could not be applied."; exit 1; fi
    echo "[ok] Agent traffic now sees ${DELAY_MS}ms +-${JITTER_MS}ms, loss ${LOSS_PERCENT}%."
    ;;
  remove|clear)
    for c in ${CONTAINERS}; do
      running "${c}" || continue
      if docker exec "${c}" tc qdisc del dev "${IFACE}" root 2>/dev/null; then
        echo "    [ok] ${c}: netem removed"
      else
        echo "    [-] ${c}: no netem rules"
      fi
    done
    ;;
  status)
    for c in ${CONTAINERS}; do
      running "${c}" || continue
      echo "--- ${c} ---"
      docker exec "${c}" tc qdisc show 2>/dev/null || echo "    (no tc rules)"
    done
    ;;
  *)
    echo "Usage: $0 [apply|remove|status] [--containers \"agent-a agent-b\"] [--interface eth0]"
    exit 1
    ;;
esac
