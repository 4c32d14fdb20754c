#!/usr/bin/env bash
# Print the running testbed's service URLs + an ssh port-forward line.
#   ./scripts/fetch_endpoints.sh [--mode single|distributed] [--json] [--ssh-target u@h]
set -euo pipefail
source "$(dirname "${BASH_SOURCE[0]}")/deploy/common.sh"
load_env
ARGS=()
while [[ $# -gt 0 ]]; do
  case "$1" in
    --mode) DEPLOYMENT_MODE="$2"; shift 2 ;;
    *) ARGS+=("$1"); shift ;;
  esac
done
FILES=(-f "$(compose_file)")
MF="$(monitoring_file)"
[[ -f "${MF}" ]] && FILES+=(-f "${MF}")
cd "${ROOT_DIR}"
py -m agentic_traffic_testing_amd.infra.endpoints "${FILES[@]}" "${ARGS[@]}"
