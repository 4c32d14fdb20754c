#!/usr/bin/env bash
# Capture inter-agent traffic to a pcap (headers only by default) with an optional
# `docker stats` JSONL side channel and a summary file.
#
#   sudo ./scripts/traffic/collect_traffic.sh [-l LABEL] [-d SECONDS] [-o DIR] [-s] [-f]
#
#   -l/--label NAME      capture label (experiment)
#   -d/--duration SECS   stop after SECS (default: until Ctrl+C)
#   -o/--output DIR      output directory (logs/traffic)
#   -s/--stats           also sample `docker stats` every 2 s
#   -f/--full-packets    full packets instead of 96-byte snaplen
#
# Outputs: packets_<label>_<ts>.pcap, stats_<label>_<ts>.jsonl, summary_<label>_<ts>.txt
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/../monitoring/lib.sh"

LABEL="experiment"; DURATION=""; OUT="${ATTA_ROOT}/logs/traffic"; STATS=false; SNAP=96
while [[ $# -gt 0 ]]; do
  case "$1" in
    -l|--label) LABEL="$2"; shift 2 ;;
    -d|--duration) DURATION="$2"; shift 2 ;;
    -o|--output) OUT="$2"; shift 2 ;;
    -s|--stats) STATS=true; shift ;;
    -f|--full-packets) SNAP=0; shift ;;
    -h|--help) sed -n '2,14p' "$0"; exit 0 ;;
    *) echo "[!] Unknown option: $1"; exit 1 ;;
  esac
done
mkdir -p "${OUT}"
TS="$(date +%Y%m%d_%H%M%S)"
PCAP="${OUT}/packets_${LABEL}_${TS}.pcap"
STATS_FILE="${OUT}/stats_${LABEL}_${TS}.jsonl"
SUMMARY="${OUT}/summary_${LABEL}_${TS}.txt"
STATS_CONTAINERS="${STATS_CONTAINERS:-agent-a agent-b agent-b-2 agent-b-3 agent-b-4 agent-b-5 llm-backend}"

[[ ${EUID} -eq 0 ]] || { echo "[!] tcpdump needs root: sudo $0 $*"; exit 1; }
command -v tcpdump >/dev/null 2>&1 || { echo "[!] tcpdump is not installed."; exit 1; }
IFACE="$(atta_find_bridge inter_agent)"
if [[ -z "${IFACE}" ]]; then
  echo "[!] inter_agent bridge not found (distributed mode not running?); using 'any'"
  IFACE=any
fi
FILTER="net ${INTER_AGENT_SUBNET}"

TCPDUMP_PID=""; STATS_PID=""
summary() {
  {
    echo "============================================================"
    echo "Traffic Capture Summary"
    echo "============================================================"
    echo "Label:     ${LABEL}"
    echo "Timestamp: ${TS}"
    echo "Duration:  ${DURATION:-manual (Ctrl+C)}"
    echo "Interface: ${IFACE}   Filter: ${FILTER}   Snaplen: ${SNAP}"
    if [[ -f "${PCAP}" ]]; then
      echo "Packet file: ${PCAP} ($(du -h "${PCAP}" | cut -f1))"
      command -v capinfos >/dev/null 2>&1 && capinfos -c -d -e "${PCAP}" 2>/dev/null || true
      echo "Total packets: $(tcpdump -r "${PCAP}" 2>/dev/null | wc -l)"
    fi
    echo
    echo "--- Topology (distributed mode) ---"
    echo "Agent A 172.23.0.10 | Agent B 172.23.0.20-24 | LLM 172.23.0.30 | Tool DB 172.23.0.40"
    echo
    echo "--- Analysis ---"
    echo "tcpdump -r ${PCAP} -q | head -50"
    echo "tcpdump -r ${PCAP} 'host 172.23.0.10 and host 172.23.0.30'      # A <-> LLM"
    echo "tcpdump -r ${PCAP} 'host 172.23.0.10 and net 172.23.0.20/29'    # A <-> B"
    echo "python3 scripts/traffic/analyze_traffic.py --pcap ${PCAP}"
  } > "${SUMMARY}"
  cat "${SUMMARY}"
}
cleanup() {
  [[ -n "${TCPDUMP_PID}" ]] && { kill "${TCPDUMP_PID}" 2>/dev/null || true; wait "${TCPDUMP_PID}" 2>/dev/null || true; }
  [[ -n "${STATS_PID}" ]] && { kill "${STATS_PID}" 2>/dev/null || true; wait "${STATS_PID}" 2>/dev/null || true; }
  summary
}
trap cleanup EXIT INT TERM

if ${STATS}; then
  (
    while true; do
      # shellcheck disable=SC2086
      docker stats --no-stream --format '{{json .}}' ${STATS_CONTAINERS} 2>/dev/null |
        sed "s/^/{\"time\":\"$(date -Iseconds)\",\"stats\":/; s/\$/}/" >> "${STATS_FILE}" || true
      sleep 2
    done
  ) &
  STATS_PID=$!
fi
echo "[*] Capturing on ${IFACE} (${FILTER}) -> ${PCAP}"
if [[ -n "${DURATION}" ]]; then
  timeout "${DURATION}" tcpdump -i "${IFACE}" -w "${PCAP}" -s "${SNAP}" ${FILTER} &
  TCPDUMP_PID=$!
  wait "${TCPDUMP_PID}" || true
  TCPDUMP_PID=""
else
  tcpdump -i "${IFACE}" -w "${PCAP}" -s "${SNAP}" ${FILTER} &
  TCPDUMP_PID=$!
  wait "${TCPDUMP_PID}" || true
  TCPDUMP_PID=""
fi
