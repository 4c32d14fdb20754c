#!/usr/bin/env bash
# Forward the testbed's web ports from a remote host over ssh.
#   ./scripts/dev/forward_clean_ssh.sh user@host [ports...]
# Local listeners on those ports that are earlier ssh forwards are closed first; any
# other process holding a port makes the script stop instead of killing it.
set -euo pipefail
TARGET="${1:?usage: $0 user@host [ports...]}"; shift || true
PORTS=("$@")
[[ ${#PORTS[@]} -eq 0 ]] && PORTS=(3000 3001 8000 8101 8102 9090 16686)
for p in "${PORTS[@]}"; do
  for pid in $(lsof -ti "tcp:${p}" -sTCP:LISTEN 2>/dev/null || true); do
    if [[ "$(ps -p "${pid}" -o comm= 2>/dev/null)" == "ssh" ]]; then
      echo "[*] closing old ssh forward on :${p} (pid ${pid})"; kill "${pid}" || true
    else
      echo "[!] port ${p} is used by pid ${pid} ($(ps -p "${pid}" -o comm=)); free it first"; exit 1
    fi
  done
done
ARGS=()
for p in "${PORTS[@]}"; do ARGS+=(-L "${p}:localhost:${p}"); done
echo "[*] ssh -N ${ARGS[*]} ${TARGET}"
exec ssh -N "${ARGS[@]}" "${TARGET}"
