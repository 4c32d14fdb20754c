#!/usr/bin/env bash
# Capture the inter-agent bridge with tcpdump and pipe it into the TCP metrics collector
# (--read-stdin), exporting tcp_* on :${PORT}.
#
# Differences from the reference script: the bridge is
# auto-detected (or --interface / TCPDUMP_INTERFACE) instead of a hard-coded br-<id>, the
# pipeline is started once, and only a previous *collector* on the port is stopped.
#
# Usage: ./scripts/monitoring/run_tcpdump.sh [--interface br-xxxx] [--port 9100]
#                                           [--filter "tcp and net 172.23.0.0/24"]
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/lib.sh"

PORT="${TCP_METRICS_PORT:-9100}"
INTERFACE="${TCPDUMP_INTERFACE:-}"
FILTER="tcp and net ${INTER_AGENT_SUBNET}"
while [[ $# -gt 0 ]]; do
  case "$1" in
    -i|--interface) INTERFACE="$2"; shift 2 ;;
    -p|--port) PORT="$2"; shift 2 ;;
    -f|--filter) FILTER="$2"; shift 2 ;;
    -h|--help) sed -n '2,11p' "$0"; exit 0 ;;
    *) echo "[run_tcpdump] unknown option: $1" >&2; exit 1 ;;
  esac
done
[[ -z "${INTERFACE}" ]] && INTERFACE="$(atta_find_bridge inter_agent)"
if [[ -z "${INTERFACE}" ]]; then
  echo "[run_tcpdump] inter-agent bridge not found; capturing on 'any'"
  INTERFACE=any
fi
echo "[run_tcpdump] interface=${INTERFACE} filter='${FILTER}' port=${PORT}"

# stop a previous collector on the port (never an unrelated process)
if command -v ss >/dev/null 2>&1; then
  for pid in $(ss -ltnpH "sport = :${PORT}" 2>/dev/null | sed -nE 's/.*pid=([0-9]+).*/\1/p' | sort -u); do
    if tr '\0' ' ' < "/proc/${pid}/cmdline" 2>/dev/null | grep -q "tcp_metrics_collector\|tcp_collector"; then
      echo "[run_tcpdump] stopping previous collector PID ${pid}"
      kill "${pid}" || true
    else
      echo "[run_tcpdump] port ${PORT} is held by PID ${pid} (not a collector); aborting" >&2
      exit 1
    fi
  done
  sleep 1
fi

cd "${ATTA_ROOT}"
# shellcheck disable=SC2086
sudo tcpdump -i "${INTERFACE}" -l -n -tt ${FILTER} \
  | "$(atta_python)" scripts/monitoring/tcp_metrics_collector.py --read-stdin --port "${PORT}"
