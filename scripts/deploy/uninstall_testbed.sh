#!/usr/bin/env bash
# Remove the testbed from this host: stop everything, remove the known
# containers, optionally wipe logs, and release GPU memory held by leftover LLM processes.
# GPU cleanup uses amd-smi / rocm-smi (the reference used nvidia-smi - Appendix B item 13)
# and only ever signals processes whose command line is this testbed's LLM server.
#   ./scripts/deploy/uninstall_testbed.sh [--keep-logs] [--yes]
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
load_env
KEEP_LOGS=0; YES=0
while [[ $# -gt 0 ]]; do
  case "$1" in
    --keep-logs) KEEP_LOGS=1; shift ;;
    --yes|-y) YES=1; shift ;;
    *) echo "[!] unknown option $1"; exit 1 ;;
  esac
done
if [[ "${YES}" != "1" ]]; then
  read -r -p "Remove all testbed containers, volumes and networks? [y/N] " ans
  [[ "${ans}" =~ ^[Yy]$ ]] || exit 0
fi
"${ROOT_DIR}/scripts/deploy/stop.sh" --all || true
for c in llm-backend agent-a agent-b agent-b-2 agent-b-3 agent-b-4 agent-b-5 mcp-tool-db chat-ui \
         jaeger prometheus grafana cadvisor cadvisor-host docker-mapping-exporter ebpf-exporter; do
  docker rm -f "${c}" >/dev/null 2>&1 && echo "[*] removed ${c}" || true
done

echo "[*] GPU processes (testbed LLM servers only):"
if command -v amd-smi >/dev/null 2>&1; then
  amd-smi process 2>/dev/null | sed 's/^/    /' || true
elif command -v rocm-smi >/dev/null 2>&1; then
  rocm-smi --showpids 2>/dev/null | sed 's/^/    /' || true
fi
for pid in $(pgrep -f "llm.serve_llm|agentic_traffic_testing_amd.serving" 2>/dev/null || true); do
  [[ "${pid}" == "$$" ]] && continue
  echo "[*] stopping LLM server pid ${pid}"
  kill "${pid}" 2>/dev/null || true
done

if [[ "${KEEP_LOGS}" != "1" ]]; then
  rm -rf "${ROOT_DIR}/logs"/* 2>/dev/null || true
  echo "[*] logs wiped"
fi
echo "[ok] uninstalled"
