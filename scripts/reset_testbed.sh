#!/usr/bin/env bash
# Full reset: uninstall, then deploy again with the same mode.
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
"${ROOT}/scripts/deploy/uninstall_testbed.sh" --yes "$@"
"${ROOT}/scripts/deploy/deploy.sh"
