#!/usr/bin/env bash
# Start the BCC eBPF TCP tools (tcpconnect, tcplife, tcprtt, tcpretrans) in the
# background on THIS node, logging under logs/<ts>_<NODE_NAME>/ (SURVEY §2.2 O9).
# Tools missing on the host are skipped; PIDs are written to pids.txt so
# `kill $(cat logs/<dir>/pids.txt)` stops exactly what this script started.
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
NODE_NAME="${NODE_NAME:-node_unspecified}"
DIR="${ROOT}/logs/$(date +%Y%m%d_%H%M%S)_${NODE_NAME}"
mkdir -p "${DIR}"
echo "[*] eBPF TCP collectors for node '${NODE_NAME}' -> ${DIR}"
for tool in tcpconnect tcplife tcprtt tcpretrans; do
  bin="$(command -v "${tool}" || command -v "${tool}-bpfcc" || true)"
  if [[ -z "${bin}" ]]; then echo "[!] ${tool} not found; skipping."; continue; fi
  sudo "${bin}" > "${DIR}/${tool}.log" 2>&1 &
  echo "$!" >> "${DIR}/pids.txt"
  echo "[*] ${tool} (pid $!) -> ${DIR}/${tool}.log"
done
echo "[*] Stop with: kill \$(cat ${DIR}/pids.txt)"
