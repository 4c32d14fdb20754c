#!/usr/bin/env bash
# One-shot crash check for cron (*/5): restart a dead, unfinished experiment in resume mode.
set -euo pipefail
ROOT="$(cd "$(dirname "${BASH_SOURCE[0]}")/../.." && pwd)"
cd "${ROOT}"
exec python3 -m agentic_traffic_testing_amd.experiments.supervise check "$@"
