#!/usr/bin/env bash
# Shared helpers for deploy / stop / uninstall / reset.
ROOT_DIR="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
COMPOSE_DIR="${ROOT_DIR}/infra"
ENV_FILE="${COMPOSE_DIR}/.env"

load_env() {
  if [[ -f "${ENV_FILE}" ]]; then
    set -a
    # shellcheck disable=SC1090
    source <(grep -Ev '^\s*(#|$)' "${ENV_FILE}")
    set +a
  fi
  DEPLOYMENT_MODE="${DEPLOYMENT_MODE:-single}"
}

compose_file() {
  case "${1:-${DEPLOYMENT_MODE}}" in
    single|multi-vm) echo "${COMPOSE_DIR}/docker-compose.yml" ;;
    distributed) echo "${COMPOSE_DIR}/docker-compose.distributed.yml" ;;
    *) echo "[!] Unknown DEPLOYMENT_MODE '${1:-${DEPLOYMENT_MODE}}' (single|distributed|multi-vm)" >&2; return 1 ;;
  esac
}

monitoring_file() {
  if [[ "${1:-${DEPLOYMENT_MODE}}" == "distributed" ]]; then
    echo "${COMPOSE_DIR}/docker-compose.monitoring.distributed.yml"
  else
    echo "${COMPOSE_DIR}/docker-compose.monitoring.yml"
  fi
}

require_docker() {
  command -v docker >/dev/null 2>&1 || { echo "[!] docker is not installed or not on PATH."; exit 1; }
  docker compose version >/dev/null 2>&1 || { echo "[!] docker compose v2 is required."; exit 1; }
}

py() { if command -v python3 >/dev/null 2>&1; then python3 "$@"; else python "$@"; fi; }

# Poll an HTTP URL until it answers 2xx (default 600 s, every 5 s).
wait_http() {
  local url="$1" timeout="${2:-600}" every="${3:-5}" t0
  t0="$(date +%s)"
  echo "[*] Waiting for ${url} (model load can take minutes)..."
  until py -c "import urllib.request,sys; urllib.request.urlopen('${url}', timeout=2).read()" >/dev/null 2>&1; do
    if (( $(date +%s) - t0 >= timeout )); then echo "[!] Timed out waiting for ${url}"; return 1; fi
    echo "    ... $(( $(date +%s) - t0 ))s"
    sleep "${every}"
  done
  echo "[*] ${url} is up."
}
