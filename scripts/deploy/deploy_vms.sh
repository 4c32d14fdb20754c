#!/usr/bin/env bash
# Create the multi-VM topology with Vagrant (infra/Vagrantfile) - SURVEY §2.2 I5.
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
command -v vagrant >/dev/null 2>&1 || { echo "[!] vagrant is not installed"; exit 1; }
cd "${ROOT}/infra"
vagrant up "$@"
vagrant status
echo "[ok] set DEPLOYMENT_MODE=multi-vm and NODE*_HOST in infra/.env, then scripts/deploy/deploy.sh"
