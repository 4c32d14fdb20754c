#!/usr/bin/env bash
# (Re)start only the UI container.  Single-host: compose service chat-ui;
# multi-host: run it on NODE1_HOST pointing the pages at Agent A there.
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/common.sh"
load_env
require_docker
if [[ "${DEPLOYMENT_MODE}" == "multi-vm" && -n "${NODE1_HOST:-}" ]]; then
  ssh "${SSH_USER:-$USER}@${NODE1_HOST}" "cd ${REMOTE_REPO_DIR:-/opt/agentic-traffic-testing}/infra && docker compose -f docker-compose.yml up -d --build --no-deps chat-ui"
else
  docker compose -f "$(compose_file)" up -d --build --no-deps chat-ui
fi
echo "[ok] UI on :3000 (/chat/, /agentverse/)"
