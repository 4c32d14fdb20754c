#!/usr/bin/env bash
# Destroy the Vagrant VMs created by deploy_vms.sh.
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
command -v vagrant >/dev/null 2>&1 || { echo "[!] vagrant is not installed"; exit 1; }
cd "${ROOT}/infra"
vagrant destroy -f "$@"
